// Host-side launcher declarations (C++ ABI, pointers as uintptr_t, stream as uintptr_t).
// Every launcher validates the shapes its grid assumes before launching.
#pragma once
#include <stdint.h>
#include <stdexcept>
#include <string>

namespace dllm {

void rms_norm(uintptr_t y, uintptr_t x, uintptr_t residual, uintptr_t w, int rows, int hidden, float eps,
              uintptr_t stream);
void rms_norm_q8(uintptr_t y, uintptr_t x, uintptr_t residual, uintptr_t w, int rows, int hidden, float eps,
                 uintptr_t q8, uintptr_t qs, uintptr_t stream);
void splitk_add_rms_norm_q8(uintptr_t y, uintptr_t residual, uintptr_t ws, int S, int M, int N, uintptr_t w,
                            float eps, uintptr_t q8, uintptr_t qs, uintptr_t stream);
void embedding(uintptr_t out, uintptr_t ids, uintptr_t table, int tokens, int hidden, int vocab,
               uintptr_t stream);
void rope_cache_append(uintptr_t q_out, uintptr_t qkv, uintptr_t positions, uintptr_t cos_sin,
                       uintptr_t k_cache, uintptr_t v_cache, uintptr_t slots, int tokens, int hq, int hkv,
                       int d, int bs, int v_groups, uintptr_t stream);
void silu_mul(uintptr_t out, uintptr_t gu, int tokens, int inter, uintptr_t stream);
void add_inplace(uintptr_t a, uintptr_t b, long n, uintptr_t stream);
void argmax(uintptr_t out, uintptr_t logits, int rows, int vocab, long row_stride, uintptr_t stream);

void splitk_add_rms_norm(uintptr_t y, uintptr_t residual, uintptr_t ws, int S, int M, int N, uintptr_t w, float eps,
                         uintptr_t stream);
void splitk_reduce(uintptr_t out, uintptr_t ws, uintptr_t bias, int S, int M, int N, uintptr_t stream);
void splitk_reduce_ex(uintptr_t out, uintptr_t ws, uintptr_t bias, int S, int M, int N, int swiglu,
                      uintptr_t stream);
int gemm_wide(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
              int mode, int variant, uintptr_t stream);
int gemm_wide_fp8(uintptr_t c, uintptr_t a, uintptr_t a_scale, uintptr_t b, uintptr_t b_scale, uintptr_t ws,
                  long ws_floats, int M, int N, int K, int splits, int mode, int variant, uintptr_t stream);
void quant_fp8_rows(uintptr_t q, uintptr_t scale, uintptr_t x, int M, int K, uintptr_t stream);
int gemm_pp(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
            int mode, int variant, uintptr_t stream);
void gemm_pp_moe(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets, int E,
                 int N, int K, int xrows, int slots, int mode, uintptr_t stream);
void gemm_pf(uintptr_t c, uintptr_t a, uintptr_t b, int M, int N, int K, int mode, int variant, uintptr_t stream);
int gemm_sq(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
            int mode, int variant, uintptr_t stream);

void moe_route(uintptr_t logits, int T, int E, int k, uintptr_t topk_w, uintptr_t topk_ids, uintptr_t counts,
               uintptr_t offsets, uintptr_t sorted_tok, uintptr_t inv, uintptr_t stream);
void moe_grouped_gemm(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets,
                      int E, int N, int K, int mode, int rows_hint, int variant, uintptr_t stream);
void moe_router_route(uintptr_t x, uintptr_t w, int T, int H, int E, int k, uintptr_t topk_w, uintptr_t topk_ids,
                      uintptr_t counts, uintptr_t offsets, uintptr_t sorted_tok, uintptr_t inv, uintptr_t stream);
void moe_wide_gemm(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets,
                   int E, int N, int K, int mode, uintptr_t stream);
void moe_wide_gemm_fp8(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets,
                       int E, int N, int K, int mode, uintptr_t sa, uintptr_t wscale, uintptr_t stream);
void moe_combine(uintptr_t out, uintptr_t ysorted, uintptr_t topk_w, uintptr_t inv, int T, int H, int k,
                 uintptr_t stream);

void paged_attention_decode(uintptr_t out, uintptr_t q, uintptr_t k_cache, uintptr_t v_cache,
                            uintptr_t block_tables, uintptr_t seq_lens, uintptr_t part_o, uintptr_t part_ml,
                            int batch, int hq, int hkv, int d, int block_size, int max_blocks, int num_splits,
                            int split_len, float scale, uintptr_t stream);
void paged_attention_decode_rope(uintptr_t out, uintptr_t qkv, uintptr_t positions, uintptr_t cos_sin, uintptr_t slots,
                                 uintptr_t k_cache, uintptr_t v_cache, uintptr_t block_tables, uintptr_t seq_lens,
                                 uintptr_t part_o, uintptr_t part_ml, int batch, int hq, int hkv, int d,
                                 int block_size, int max_blocks, int num_splits, int split_len, float scale,
                                 uintptr_t qkv_part, int qkv_nparts, long qkv_slab, uintptr_t stream);
void paged_attention_prefill(uintptr_t out, uintptr_t q, uintptr_t k_cache, uintptr_t v_cache,
                             uintptr_t block_tables, uintptr_t cu_seqlens_q, uintptr_t seq_lens, int batch,
                             int hq, int hkv, int d, int block_size, int max_blocks, int max_q_len, float scale,
                             int version, uintptr_t positions, uintptr_t cos_sin, int q_stride, uintptr_t stream);

long p2p_inbox_bytes(long chunk, int nslots);
void p2p_standin(uintptr_t src, uintptr_t s_inbox, long s_bytes, uint64_t s_seq0, uintptr_t dst, uintptr_t r_inbox,
                 long r_bytes, uint64_t r_seq0, long chunk, int nslots, int channels, uintptr_t abort_word,
                 double timeout_s, uintptr_t err, int lds_bytes, uintptr_t stream);
uintptr_t p2p_host_words(int n);
void p2p_host_words_free(uintptr_t p);

}  // namespace dllm
