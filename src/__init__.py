"""Compatibility namespace with the reference layout (``src.master``, ``src.worker``,
``src.network``, ``src.model``).  Everything lives in :mod:`distributed_llms_amd`; these
modules re-export it so code written against the reference's import paths keeps working.
"""
