"""In-tree build of the native extensions (no torch JIT cache, no hipify).

    python -m distributed_llms_amd.csrc.build [--force] [-j N]

* ``_C_kernels``: every ``csrc/kernels/*.hip`` compiled by ``hipcc --offload-arch=gfx950``
  plus the pybind11 binding TU, linked into ``distributed_llms_amd/_C_kernels<EXT_SUFFIX>``.
* ``_C_runtime``: host-only C++17 (``csrc/runtime/*.cpp``), paged-KV block manager and
  wire-frame codec, linked into ``distributed_llms_amd/_C_runtime<EXT_SUFFIX>``.
* ``_C_rccl``: native RCCL p2p transport (``csrc/comm/rccl_p2p.cpp``) and the HIP-IPC
  peer-write data plane (``csrc/comm/ipc_p2p.cpp``), linked against ``librccl.so.1`` -- at run
  time the copy PyTorch already loaded (one RCCL per process).

Objects go to ``build/`` (git-ignored); the ``.so`` files land in the package
directory so they travel to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("DLLM_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


# per-source extra flags.  attention.hip: its softmax takes fmaxf of MFMA results and of
# v_permlane swap results, which hipcc (IEEE mode) first quiets with a v_max_f32 x, x, x each --
# 56 of the prefill loop's 88 max instructions; the kernels never produce a NaN (masked scores are
# -inf and every subtraction keeps a finite reference), so NaN semantics are dropped for that file
FILE_FLAGS = {"attention.hip": ["-fno-honor-nans"]}


def kernel_flags(src: str):
    """hipcc flags of one csrc/kernels source (without includes / output)."""
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
              "-mcode-object-version=5"]
    if os.environ.get("DLLM_PART_TYPE"):        # split-K slab type (common.h); rebuild with force=True
        common.append(f"-DDLLM_PART_TYPE={int(os.environ['DLLM_PART_TYPE'])}")
    return common + FILE_FLAGS.get(os.path.basename(src), [])


def _py_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _ext_path(name: str) -> str:
    return os.path.join(PKG, name + sysconfig.get_config_var("EXT_SUFFIX"))


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _link(cmd_prefix, target, rest):
    """Link into a temporary file, then rename over the target: a process importing the module
    meanwhile (or a snapshot of the tree) never sees a half-written .so."""
    tmp = target + ".tmp"
    _run(cmd_prefix + ["-o", tmp] + rest)
    os.replace(tmp, target)


def build_kernels(force=False, jobs=8, verbose=False) -> str:
    src_dir = os.path.join(HERE, "kernels")
    out_dir = os.path.join(BUILD, "kernels")
    os.makedirs(out_dir, exist_ok=True)
    headers = glob.glob(os.path.join(src_dir, "*.h"))
    hips = sorted(glob.glob(os.path.join(src_dir, "*.hip")))
    incs = [f"-I{p}" for p in _py_includes()] + [f"-I{src_dir}"]
    jobs_list = []
    objs = []
    for src in hips:
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + headers + [os.path.abspath(__file__)]):
            jobs_list.append([HIPCC, "-c", src, "-o", obj] + kernel_flags(src) + incs)
    bind = os.path.join(src_dir, "bindings.cpp")
    bobj = os.path.join(out_dir, "bindings.o")
    objs.append(bobj)
    if force or _stale(bobj, [bind] + headers):
        jobs_list.append([CXX, "-c", bind, "-o", bobj, "-O2", "-std=c++17", "-fPIC",
                          "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__"] + incs)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)
    target = _ext_path("_C_kernels")
    if force or _stale(target, objs):
        _link([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"], target, objs)
    return target


def build_runtime(force=False, jobs=8, verbose=False) -> str:
    src_dir = os.path.join(HERE, "runtime")
    out_dir = os.path.join(BUILD, "runtime")
    os.makedirs(out_dir, exist_ok=True)
    headers = glob.glob(os.path.join(src_dir, "*.h"))
    srcs = sorted(glob.glob(os.path.join(src_dir, "*.cpp")))
    incs = [f"-I{p}" for p in _py_includes()] + [f"-I{src_dir}"]
    objs, jobs_list = [], []
    for src in srcs:
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + headers):
            jobs_list.append([CXX, "-c", src, "-o", obj, "-O2", "-std=c++17", "-fPIC",
                              "-fvisibility=hidden", "-Wall"] + incs)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(_run, jobs_list))
    target = _ext_path("_C_runtime")
    if force or _stale(target, objs):
        _link([CXX, "-shared", "-fPIC"], target, objs)
    return target


def build_runtime_sanitized(out_dir: str) -> str:
    """The host runtime (``_C_runtime``: block manager, frame codec) built with UBSan
    (-fsanitize=undefined, no recovery, runtime linked statically so the module loads into a plain
    interpreter) and libstdc++ assertions (container bounds) -- SURVEY §5.2's sanitizer build.
    ASan would need the interpreter started with libasan preloaded; UBSan + _GLIBCXX_ASSERTIONS
    catch out-of-bounds indexing, overflow and misaligned access in-process.  Returns the .so path
    (import it under the name ``distributed_llms_amd._C_runtime``)."""
    src_dir = os.path.join(HERE, "runtime")
    os.makedirs(out_dir, exist_ok=True)
    target = os.path.join(out_dir, os.path.basename(_ext_path("_C_runtime")))
    _run([CXX, "-shared", "-fPIC", "-O1", "-g", "-std=c++17", "-fvisibility=hidden",
          "-fsanitize=undefined", "-fno-sanitize-recover=undefined", "-static-libubsan", "-D_GLIBCXX_ASSERTIONS",
          *[f"-I{p}" for p in _py_includes()], f"-I{src_dir}",
          *sorted(glob.glob(os.path.join(src_dir, "*.cpp"))), "-o", target])
    return target


def build_comm(force=False, jobs=8, verbose=False) -> str:
    out_dir = os.path.join(BUILD, "comm")
    os.makedirs(out_dir, exist_ok=True)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    objs = []
    for name in ("rccl_p2p", "ipc_p2p"):
        src = os.path.join(HERE, "comm", name + ".cpp")
        obj = os.path.join(out_dir, name + ".o")
        objs.append(obj)
        if force or _stale(obj, [src]):
            _run([CXX, "-c", src, "-o", obj, "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
                  "-D__HIP_PLATFORM_AMD__", f"-I{rocm}/include"] + [f"-I{p}" for p in _py_includes()])
    target = _ext_path("_C_rccl")
    if force or _stale(target, objs):
        _link([CXX, "-shared", "-fPIC"], target, [*objs, f"-L{rocm}/lib", "-lrccl", "-lamdhip64"])
    return target


def build_all(force=False, jobs=8, verbose=False):
    return build_runtime(force, jobs, verbose), build_kernels(force, jobs, verbose), build_comm(force, jobs, verbose)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--only", choices=["kernels", "runtime", "comm"], default=None)
    a = ap.parse_args(argv)
    if a.only in (None, "runtime"):
        print("built", build_runtime(a.force, a.jobs, a.verbose))
    if a.only in (None, "kernels"):
        print("built", build_kernels(a.force, a.jobs, a.verbose))
    if a.only in (None, "comm"):
        print("built", build_comm(a.force, a.jobs, a.verbose))


if __name__ == "__main__":
    sys.exit(main())
