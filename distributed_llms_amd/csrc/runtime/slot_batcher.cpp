// Native decode-step bookkeeping for the continuous-batching scheduler (engine/scheduler.py).
//
// The reference has no generation loop; its per-request state is a Python
// dict touched from several threads (D21).  Here the hot part of the scheduler -- the running
// sequences of every microbatch slot, their lengths / last tokens / stop conditions and the
// decode batch metadata -- lives in this class, next to the paged-KV BlockManager it allocates
// from.  Per decode microbatch the driver makes two calls:
//
//   build_decode(slot, ...) -> the packed int32 batch (HostBatch wire format, engine/batch.py),
//                              block tables and slot mappings written straight from the tables
//   complete(slot, rows, tokens, now) -> append sampled ids, apply EOS / length / max_seq_len
//
// instead of ~900 us of per-sequence Python at batch 256 (bench/host_overhead.py), which would
// make the pipeline's stage 0 host-bound at 8 stages (a stage's GPU time per microbatch is
// ~0.9 ms there).  Python Sequence objects are synced only when a sequence leaves the running
// set (finished, preempted, aborted): take_finished() / take_preempted() + take_output().
//
// Lookahead (build_decode(..., lookahead=true)): the next decode step of a slot is built while
// `pend` earlier steps of its sequences are still in flight; their input ids come from the
// device, so the packed ids are placeholders, and sequences that finish by length within the
// pending steps are left out.  A sequence finishing by EOS in a pending step costs one
// throw-away row: complete() skips rows of sequences that are no longer running.
#include "block_manager.h"

#include <pybind11/stl.h>

#include <string>

namespace {

constexpr int HDR = 16;   // HostBatch.pack header length (engine/batch.py)

enum Reason : int { R_NONE = 0, R_EOS = 1, R_LENGTH = 2, R_MAX_SEQ = 3, R_ABORT = 4 };

struct SeqRec {
  int slot = 0;
  int32_t len = 0;        // tokens whose values the host knows (prompt + completed outputs)
  int32_t pend = 0;       // decode steps issued for it and not completed yet
  int32_t remaining = 0;  // tokens still to generate
  int32_t eos = -1;       // < 0: no EOS stop
  int32_t last = 0;       // newest known token
  int32_t samp[3] = {0, 0, 10000};   // temperature * 1e4, top_k, top_p * 1e4
  bool running = true;
  int reason = R_NONE;
  std::vector<int32_t> out;     // tokens generated while registered here
  std::vector<double> times;    // their host completion timestamps
};

}  // namespace

class SlotBatcher {
 public:
  SlotBatcher(BlockManager& bm, int num_slots, int max_seq_len)
      : bm_(bm), order_(std::max(1, num_slots)), last_rows_(std::max(1, num_slots)), max_seq_len_(max_seq_len) {
    if (max_seq_len < 2) throw std::invalid_argument("max_seq_len must be >= 2");
  }

  int num_slots() const { return (int)order_.size(); }
  int max_seq_len() const { return max_seq_len_; }

  // Register a sequence that finished its prefill and keeps decoding in `slot`.
  void admit(int slot, int64_t id, int32_t len, int32_t last, int32_t remaining, int32_t eos, int32_t temp_e4,
             int32_t top_k, int32_t top_p_e4) {
    check_slot(slot);
    if (recs_.count(id)) throw std::invalid_argument("sequence already registered");
    if (remaining <= 0 || len >= max_seq_len_ || len < 1) throw std::invalid_argument("admit: nothing to decode");
    SeqRec r;
    r.slot = slot;
    r.len = len;
    r.last = last;
    r.remaining = remaining;
    r.eos = eos;
    r.samp[0] = temp_e4;
    r.samp[1] = top_k;
    r.samp[2] = top_p_e4;
    recs_.emplace(id, std::move(r));
    order_[slot].push_back(id);
  }

  int num_running(int slot) const {
    check_slot(slot);
    return (int)order_[slot].size();
  }

  int num_running_total() const {
    size_t n = 0;
    for (const auto& o : order_) n += o.size();
    return (int)n;
  }

  int min_running() const {
    size_t n = order_[0].size();
    for (const auto& o : order_) n = std::min(n, o.size());
    return (int)n;
  }

  py::array_t<int64_t> running_ids(int slot) const {
    check_slot(slot);
    const auto& o = order_[slot];
    py::array_t<int64_t> a((py::ssize_t)o.size());
    std::copy(o.begin(), o.end(), a.mutable_data());
    return a;
  }

  // (len, pend, remaining) of a registered sequence (tests / diagnostics)
  py::tuple state(int64_t id) const {
    const SeqRec& r = rec(id);
    return py::make_tuple(r.len, r.pend, r.remaining, r.running);
  }

  // Build the slot's next decode step.  Returns None when there is nothing to run (or, with
  // lookahead, when the step cannot be built without the host: a capacity failure or a row the
  // newest step of the slot did not carry).  Otherwise (packed int32 batch, rows int64 seq ids,
  // keep) with keep = positions of the rows in the slot's previous step (lookahead) or None.
  // Synchronous mode preempts the youngest sequences of the slot until the KV cache fits.
  py::object build_decode(int slot, int max_blocks, int step_id, bool lookahead) {
    check_slot(slot);
    if (max_blocks < 1) throw std::invalid_argument("max_blocks >= 1");
    auto& ord = order_[slot];
    std::vector<int64_t> rows;
    rows.reserve(ord.size());
    std::vector<int64_t> keep;
    if (!lookahead) {
      size_t i = 0;
      while (i < ord.size()) {
        SeqRec& r = rec(ord[i]);
        if (r.pend != 0) throw std::logic_error("synchronous decode step with a step still in flight");
        if (bm_.ensure_capacity(ord[i], r.len)) {
          ++i;
          continue;
        }
        preempt_youngest(slot);     // may remove ord[i] itself; the loop re-checks the bound
      }
      rows.assign(ord.begin(), ord.end());
    } else {
      const auto& prev = last_rows_[slot];
      std::unordered_map<int64_t, int64_t> pos;
      pos.reserve(prev.size() * 2);
      for (size_t j = 0; j < prev.size(); ++j) pos.emplace(prev[j], (int64_t)j);
      for (int64_t id : ord) {
        const SeqRec& r = rec(id);
        if (r.remaining - r.pend <= 0 || r.len + r.pend >= max_seq_len_) continue;   // done by length
        auto it = pos.find(id);
        if (it == pos.end()) return py::none();
        if (!bm_.ensure_capacity(id, r.len + r.pend)) return py::none();
        rows.push_back(id);
        keep.push_back(it->second);
      }
    }
    if (rows.empty()) return py::none();

    const int b = (int)rows.size();
    bool has_s = false;
    for (int64_t id : rows) has_s |= rec(id).samp[0] > 0;
    const size_t n = HDR + 3 * (size_t)b + b + (b + 1) + (size_t)b * max_blocks + b + (has_s ? 3 * (size_t)b : 0);
    py::array_t<int32_t> packed((py::ssize_t)n);
    int32_t* p = packed.mutable_data();
    std::fill(p, p + HDR, 0);
    int32_t* ids = p + HDR;
    int32_t* positions = ids + b;
    int32_t* slots = positions + b;
    int32_t* seq_lens = slots + b;
    int32_t* cu = seq_lens + b;
    int32_t* bt = cu + b + 1;
    int32_t* lidx = bt + (size_t)b * max_blocks;
    int32_t* samp = lidx + b;
    const int bs = bm_.block_size();
    int32_t max_ctx = 0;
    for (int i = 0; i < b; ++i) {
      SeqRec& r = rec(rows[i]);
      const int32_t ctx = r.len + r.pend;          // tokens in the context after this step's append
      const int32_t pos_i = ctx - 1;               // this step's input token position
      const std::vector<int32_t>* t = bm_.table(rows[i]);
      if (!t || (int)t->size() * bs < ctx) throw std::logic_error("KV capacity missing for a decode row");
      if ((int)t->size() > max_blocks) throw std::invalid_argument("sequence has more blocks than max_blocks");
      ids[i] = r.pend == 0 ? r.last : 0;
      positions[i] = pos_i;
      slots[i] = (*t)[pos_i / bs] * bs + pos_i % bs;
      seq_lens[i] = ctx;
      cu[i] = i;
      int32_t* row = bt + (size_t)i * max_blocks;
      std::copy(t->begin(), t->end(), row);
      std::fill(row + t->size(), row + max_blocks, 0);
      lidx[i] = i;
      if (has_s) std::copy(r.samp, r.samp + 3, samp + 3 * (size_t)i);
      max_ctx = std::max(max_ctx, ctx);
      r.pend += 1;
    }
    cu[b] = b;
    p[0] = 0;            // decode
    p[1] = b;            // tokens
    p[2] = b;            // sequences
    p[3] = max_blocks;
    p[4] = 1;            // max_q_len
    p[5] = max_ctx;
    p[6] = slot;
    p[7] = step_id;
    p[8] = has_s ? 1 : 0;

    py::array_t<int64_t> rows_a(b);
    std::copy(rows.begin(), rows.end(), rows_a.mutable_data());
    py::object keep_o = py::none();
    if (lookahead && keep.size() != last_rows_[slot].size()) {
      py::array_t<int64_t> k((py::ssize_t)keep.size());
      std::copy(keep.begin(), keep.end(), k.mutable_data());
      keep_o = k;
    }
    last_rows_[slot] = std::move(rows);
    return py::make_tuple(packed, rows_a, keep_o);
  }

  // Apply the sampled ids of a decode step (rows as returned by build_decode).  Returns how many
  // sequences finished; take_finished() lists them.
  int complete(int slot, py::array_t<int64_t, py::array::c_style | py::array::forcecast> rows,
               py::array_t<int32_t, py::array::c_style | py::array::forcecast> tokens, double now) {
    check_slot(slot);
    auto rw = rows.unchecked<1>();
    auto tk = tokens.unchecked<1>();
    if (tk.shape(0) < rw.shape(0)) throw std::invalid_argument("fewer tokens than rows");
    int nfin = 0;
    for (py::ssize_t i = 0; i < rw.shape(0); ++i) {
      auto it = recs_.find(rw(i));
      if (it == recs_.end()) continue;          // finished (or aborted) and already taken
      SeqRec& r = it->second;
      if (!r.running) continue;                  // throw-away lookahead row
      if (r.pend <= 0) throw std::logic_error("complete() for a row with no step in flight");
      const int32_t tok = tk(i);
      r.pend -= 1;
      r.len += 1;
      r.remaining -= 1;
      r.last = tok;
      r.out.push_back(tok);
      r.times.push_back(now);
      int why = R_NONE;
      if (r.eos >= 0 && tok == r.eos) why = R_EOS;
      else if (r.remaining <= 0) why = R_LENGTH;
      else if (r.len >= max_seq_len_) why = R_MAX_SEQ;
      if (why != R_NONE) {
        stop(rw(i), r, why);
        ++nfin;
      }
    }
    if (nfin) compact(slot);
    return nfin;
  }

  // Abort a registered sequence (frees its KV blocks; its tokens stay until take_output).
  bool abort(int64_t id) {
    auto it = recs_.find(id);
    if (it == recs_.end() || !it->second.running) return false;
    const int slot = it->second.slot;
    stop(id, it->second, R_ABORT);
    compact(slot);
    return true;
  }

  // [(seq id, reason)] of the sequences that stopped since the last call.
  std::vector<std::pair<int64_t, std::string>> take_finished() {
    static const char* names[] = {"", "eos", "length", "max_seq_len", "abort"};
    std::vector<std::pair<int64_t, std::string>> out;
    out.reserve(finished_.size());
    for (auto& f : finished_) out.emplace_back(f.first, names[f.second]);
    finished_.clear();
    return out;
  }

  std::vector<int64_t> take_preempted() {
    std::vector<int64_t> out;
    out.swap(preempted_);
    return out;
  }

  // (tokens int32, times float64) generated while registered; drops the record.
  py::tuple take_output(int64_t id) {
    auto it = recs_.find(id);
    if (it == recs_.end()) throw std::out_of_range("unknown sequence in take_output");
    if (it->second.running) throw std::logic_error("take_output of a running sequence");
    const SeqRec& r = it->second;
    py::array_t<int32_t> toks((py::ssize_t)r.out.size());
    py::array_t<double> times((py::ssize_t)r.times.size());
    std::copy(r.out.begin(), r.out.end(), toks.mutable_data());
    std::copy(r.times.begin(), r.times.end(), times.mutable_data());
    recs_.erase(it);
    return py::make_tuple(toks, times);
  }

  // Tokens generated so far by a running sequence (a copy; for status / streaming readers).
  py::array_t<int32_t> peek_output(int64_t id) const {
    const SeqRec& r = rec(id);
    py::array_t<int32_t> toks((py::ssize_t)r.out.size());
    std::copy(r.out.begin(), r.out.end(), toks.mutable_data());
    return toks;
  }

 private:
  void check_slot(int slot) const {
    if (slot < 0 || slot >= (int)order_.size()) throw std::out_of_range("slot out of range");
  }

  SeqRec& rec(int64_t id) {
    auto it = recs_.find(id);
    if (it == recs_.end()) throw std::out_of_range("unknown sequence");
    return it->second;
  }
  const SeqRec& rec(int64_t id) const {
    auto it = recs_.find(id);
    if (it == recs_.end()) throw std::out_of_range("unknown sequence");
    return it->second;
  }

  void stop(int64_t id, SeqRec& r, int why) {
    r.running = false;
    r.reason = why;
    bm_.free_sequence(id);
    finished_.emplace_back(id, why);
  }

  void preempt_youngest(int slot) {
    auto& ord = order_[slot];
    const int64_t id = ord.back();
    ord.pop_back();
    SeqRec& r = rec(id);
    r.running = false;
    bm_.free_sequence(id);
    preempted_.push_back(id);
  }

  void compact(int slot) {
    auto& ord = order_[slot];
    ord.erase(std::remove_if(ord.begin(), ord.end(),
                             [&](int64_t id) {
                               auto it = recs_.find(id);
                               return it == recs_.end() || !it->second.running;
                             }),
              ord.end());
  }

  BlockManager& bm_;
  std::vector<std::vector<int64_t>> order_;      // per slot, admission order (youngest last)
  std::vector<std::vector<int64_t>> last_rows_;  // per slot, rows of the newest built step
  std::unordered_map<int64_t, SeqRec> recs_;
  std::vector<std::pair<int64_t, int>> finished_;
  std::vector<int64_t> preempted_;
  int max_seq_len_;
};

void register_slot_batcher(py::module_& m) {
  py::class_<SlotBatcher>(m, "SlotBatcher")
      .def(py::init<BlockManager&, int, int>(), py::arg("block_manager"), py::arg("num_slots"),
           py::arg("max_seq_len"), py::keep_alive<1, 2>())
      .def_property_readonly("num_slots", &SlotBatcher::num_slots)
      .def_property_readonly("max_seq_len", &SlotBatcher::max_seq_len)
      .def("admit", &SlotBatcher::admit, py::arg("slot"), py::arg("seq_id"), py::arg("length"), py::arg("last_token"),
           py::arg("remaining"), py::arg("eos") = -1, py::arg("temp_e4") = 0, py::arg("top_k") = 0,
           py::arg("top_p_e4") = 10000)
      .def("num_running", &SlotBatcher::num_running)
      .def("num_running_total", &SlotBatcher::num_running_total)
      .def("min_running", &SlotBatcher::min_running)
      .def("running_ids", &SlotBatcher::running_ids)
      .def("state", &SlotBatcher::state)
      .def("build_decode", &SlotBatcher::build_decode, py::arg("slot"), py::arg("max_blocks"), py::arg("step_id") = 0,
           py::arg("lookahead") = false)
      .def("complete", &SlotBatcher::complete, py::arg("slot"), py::arg("rows"), py::arg("tokens"), py::arg("now"))
      .def("abort", &SlotBatcher::abort)
      .def("take_finished", &SlotBatcher::take_finished)
      .def("take_preempted", &SlotBatcher::take_preempted)
      .def("take_output", &SlotBatcher::take_output)
      .def("peek_output", &SlotBatcher::peek_output);
}
