// _C_runtime: host-side native runtime pieces (no HIP dependency).
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_block_manager(py::module_& m);
void register_frame_codec(py::module_& m);
void register_slot_batcher(py::module_& m);

PYBIND11_MODULE(_C_runtime, m) {
  m.doc() = "distributed_llms_amd native runtime (KV block manager, decode-slot batcher, wire-frame codec)";
  register_block_manager(m);
  register_frame_codec(m);
  register_slot_batcher(m);
}
