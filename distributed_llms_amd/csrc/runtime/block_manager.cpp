// Paged-KV block manager (host side, N4 in SURVEY §2.2).
//
// The reference keeps no KV cache at all.  Every pipeline
// stage holds the KV of ALL running sequences for ITS layers, so one block
// table per sequence is valid on every stage: the scheduler on stage 0 owns
// this manager and ships block tables with each microbatch's metadata.
//
// Blocks are handed out from a LIFO free list (recently freed blocks are the
// ones most likely still resident in the 256 MiB Infinity Cache).  All batch
// metadata (block tables, slot mappings) is written straight into numpy
// buffers so the per-step Python cost is O(1) calls.
#include "block_manager.h"

void register_block_manager(py::module_& m) {
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int>(), py::arg("num_blocks"), py::arg("block_size"))
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def("num_free", &BlockManager::num_free)
      .def("num_sequences", &BlockManager::num_sequences)
      .def("blocks_for", &BlockManager::blocks_for)
      .def("has_sequence", &BlockManager::has_sequence)
      .def("extra_blocks_needed", &BlockManager::extra_blocks_needed)
      .def("can_fit", &BlockManager::can_fit)
      .def("ensure_capacity", &BlockManager::ensure_capacity)
      .def("ensure_capacity_batch", &BlockManager::ensure_capacity_batch)
      .def("free_sequence", &BlockManager::free_sequence)
      .def("block_table", &BlockManager::block_table)
      .def("fill_block_tables", &BlockManager::fill_block_tables, py::arg("seqs"), py::arg("out"),
           py::arg("pad") = 0)
      .def("fill_slots", &BlockManager::fill_slots);
}
