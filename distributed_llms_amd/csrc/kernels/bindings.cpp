// pybind11 bindings for the gfx950 kernel launchers.
// Tensors cross the boundary as raw device pointers (uintptr_t) plus explicit
// shapes; the Python wrappers in distributed_llms_amd/ops check dtype/contiguity
// and pass torch's current HIP stream, so every launch is graph-capturable.
#include <pybind11/pybind11.h>

#include "launchers.h"

namespace py = pybind11;

PYBIND11_MODULE(_C_kernels, m) {
  m.doc() = "distributed_llms_amd HIP kernels (gfx950 / CDNA4)";
  m.attr("arch") = "gfx950";
  m.def("rms_norm", &dllm::rms_norm, py::arg("y"), py::arg("x"), py::arg("residual"), py::arg("w"),
        py::arg("rows"), py::arg("hidden"), py::arg("eps"), py::arg("stream"));
  m.def("embedding", &dllm::embedding);
  m.def("rope_cache_append", &dllm::rope_cache_append);
  m.def("silu_mul", &dllm::silu_mul);
  m.def("argmax", &dllm::argmax);
  m.def("add_inplace", &dllm::add_inplace);
  m.def("moe_route", &dllm::moe_route);
  m.def("moe_grouped_gemm", &dllm::moe_grouped_gemm);
  m.def("splitk_add_rms_norm", &dllm::splitk_add_rms_norm);
  m.def("splitk_reduce", &dllm::splitk_reduce);
  m.def("gemm_wide", &dllm::gemm_wide);
  m.def("gemm_wide_fp8", &dllm::gemm_wide_fp8);
  m.def("quant_fp8_rows", &dllm::quant_fp8_rows);
  m.def("rms_norm_q8", &dllm::rms_norm_q8);
  m.def("moe_wide_gemm_fp8", &dllm::moe_wide_gemm_fp8);
  m.def("splitk_add_rms_norm_q8", &dllm::splitk_add_rms_norm_q8);
  m.def("gemm_sq", &dllm::gemm_sq);
  m.def("gemm_pp_moe", &dllm::gemm_pp_moe);
  m.def("gemm_pp", &dllm::gemm_pp);
  m.def("gemm_pf", &dllm::gemm_pf);
  m.def("moe_combine", &dllm::moe_combine);
  m.def("moe_wide_gemm", &dllm::moe_wide_gemm);
  m.def("moe_router_route", &dllm::moe_router_route);
  m.def("paged_attention_decode", &dllm::paged_attention_decode);
  m.def("paged_attention_decode_rope", &dllm::paged_attention_decode_rope);
  m.def("paged_attention_prefill", &dllm::paged_attention_prefill);
  m.def("p2p_inbox_bytes", &dllm::p2p_inbox_bytes);
  m.def("p2p_standin", &dllm::p2p_standin);
  m.def("p2p_host_words", &dllm::p2p_host_words);
  m.def("p2p_host_words_free", &dllm::p2p_host_words_free);
}
