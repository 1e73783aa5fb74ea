// Paged-KV block manager (host side, N4 in SURVEY §2.2): the class, shared by the pybind11
// registration (block_manager.cpp) and the decode-slot batcher (slot_batcher.cpp).
#pragma once

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

class BlockManager {
 public:
  BlockManager(int num_blocks, int block_size) : num_blocks_(num_blocks), block_size_(block_size) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks/block_size must be > 0");
    free_.reserve(num_blocks);
    for (int b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  }

  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  int num_free() const { return (int)free_.size(); }
  int num_sequences() const { return (int)tables_.size(); }
  int blocks_for(int64_t tokens) const { return (int)((tokens + block_size_ - 1) / block_size_); }

  bool has_sequence(int64_t seq) const { return tables_.count(seq) != 0; }

  // Blocks a sequence still needs to hold `tokens` tokens in total.
  int extra_blocks_needed(int64_t seq, int64_t tokens) const {
    auto it = tables_.find(seq);
    const int have = it == tables_.end() ? 0 : (int)it->second.size();
    return std::max(0, blocks_for(tokens) - have);
  }

  bool can_fit(int64_t seq, int64_t tokens) const { return extra_blocks_needed(seq, tokens) <= num_free(); }

  // Direct table access for the native batcher (nullptr = unknown sequence).
  const std::vector<int32_t>* table(int64_t seq) const {
    auto it = tables_.find(seq);
    return it == tables_.end() ? nullptr : &it->second;
  }

  // Grow the sequence's table to hold `tokens` tokens. All-or-nothing.
  bool ensure_capacity(int64_t seq, int64_t tokens) {
    const int need = extra_blocks_needed(seq, tokens);
    if (need > num_free()) return false;
    auto& t = tables_[seq];
    for (int i = 0; i < need; ++i) {
      t.push_back(free_.back());
      free_.pop_back();
    }
    return true;
  }

  // Grow every sequence i to lens[i] tokens, in order; returns the index of the first one that
  // does not fit (nothing allocated for it or after it), or -1 when all fit.  One call per
  // decode step instead of one per sequence.
  int64_t ensure_capacity_batch(py::array_t<int64_t, py::array::c_style> seqs,
                                py::array_t<int64_t, py::array::c_style> lens) {
    auto s = seqs.unchecked<1>();
    auto l = lens.unchecked<1>();
    if (s.shape(0) != l.shape(0)) throw std::invalid_argument("seqs/lens length mismatch");
    for (py::ssize_t i = 0; i < s.shape(0); ++i)
      if (!ensure_capacity(s(i), l(i))) return i;
    return -1;
  }

  void free_sequence(int64_t seq) {
    auto it = tables_.find(seq);
    if (it == tables_.end()) return;
    for (auto b = it->second.rbegin(); b != it->second.rend(); ++b) free_.push_back(*b);
    tables_.erase(it);
  }

  std::vector<int32_t> block_table(int64_t seq) const {
    auto it = tables_.find(seq);
    if (it == tables_.end()) throw std::out_of_range("unknown sequence");
    return it->second;
  }

  // out[B, max_blocks] int32 (C-contiguous), rows padded with `pad`.
  void fill_block_tables(py::array_t<int64_t, py::array::c_style> seqs,
                         py::array_t<int32_t, py::array::c_style> out, int32_t pad) const {
    auto s = seqs.unchecked<1>();
    auto o = out.mutable_unchecked<2>();
    if (o.shape(0) < s.shape(0)) throw std::invalid_argument("block table buffer too small");
    const int mb = (int)o.shape(1);
    for (py::ssize_t i = 0; i < s.shape(0); ++i) {
      auto it = tables_.find(s(i));
      if (it == tables_.end()) throw std::out_of_range("unknown sequence in fill_block_tables");
      const auto& t = it->second;
      if ((int)t.size() > mb) throw std::invalid_argument("sequence has more blocks than max_blocks");
      int j = 0;
      for (; j < (int)t.size(); ++j) o(i, j) = t[j];
      for (; j < mb; ++j) o(i, j) = pad;
    }
  }

  // Slot ids for tokens [start[i], start[i]+count[i]) of each sequence, packed in order.
  int fill_slots(py::array_t<int64_t, py::array::c_style> seqs, py::array_t<int32_t, py::array::c_style> start,
                 py::array_t<int32_t, py::array::c_style> count, py::array_t<int32_t, py::array::c_style> out) const {
    auto s = seqs.unchecked<1>();
    auto st = start.unchecked<1>();
    auto ct = count.unchecked<1>();
    auto o = out.mutable_unchecked<1>();
    py::ssize_t k = 0;
    for (py::ssize_t i = 0; i < s.shape(0); ++i) {
      auto it = tables_.find(s(i));
      if (it == tables_.end()) throw std::out_of_range("unknown sequence in fill_slots");
      const auto& t = it->second;
      for (int p = st(i); p < st(i) + ct(i); ++p) {
        const int bi = p / block_size_;
        if (bi >= (int)t.size()) throw std::out_of_range("token position beyond allocated blocks");
        if (k >= o.shape(0)) throw std::invalid_argument("slot buffer too small");
        o(k++) = t[bi] * block_size_ + p % block_size_;
      }
    }
    return (int)k;
  }

 private:
  int num_blocks_;
  int block_size_;
  std::vector<int32_t> free_;
  std::unordered_map<int64_t, std::vector<int32_t>> tables_;
};

