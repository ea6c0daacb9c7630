// Native data pipeline for paddle_ray_amd.io.
//
// Parity: the reference's C++ reader / DataLoader plumbing (paddle/fluid/operators/reader/
// buffered_reader.cc: a ring of pre-fetched batches copied H2D on a side stream;
// paddle/fluid/imperative/data_loader.cc) and the GPT pretraining dataset index helpers its
// Fleet benchmarks use (sample index over concatenated documents).
//
// Pieces:
//  * build_sample_idx: (doc sizes, doc order, seq_len, epochs) -> [n+1, 2] (doc position,
//    token offset) start of every seq_len+1 token sample over the concatenated document
//    stream (samples span document boundaries; consecutive samples overlap by one token).
//  * TokenLoader: a ring of `nslots` batch buffers (host memory owned by the caller — pinned
//    torch tensors, so the H2D copy is a true async DMA) filled by `nthreads` worker threads
//    that gather [batch, seq_len+1] int64 token windows straight out of a memory-mapped token
//    file (uint16 / int32 / int64). Python acquires slot i (blocking WITHOUT the GIL), issues
//    a non_blocking copy to HBM, and releases the slot after that copy's event completed.
//  * stack_rows: multi-threaded memcpy of many equally-sized sample buffers into one batch
//    buffer (the collate of the generic DataLoader), GIL released.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace pra_data {

py::array_t<int64_t> build_sample_idx(py::array_t<int32_t, py::array::c_style | py::array::forcecast> sizes,
                                      py::array_t<int32_t, py::array::c_style | py::array::forcecast> doc_idx,
                                      int64_t seq_length, int64_t num_epochs, int64_t tokens_per_epoch) {
  const int32_t* sz = sizes.data();
  const int32_t* di = doc_idx.data();
  const int64_t ndoc_idx = doc_idx.size();
  const int64_t n_samples = (num_epochs * tokens_per_epoch - 1) / seq_length;
  py::array_t<int64_t> out({n_samples + 1, (int64_t)2});
  auto o = out.mutable_unchecked<2>();
  int64_t pos = 0;     // index into doc_idx
  int64_t offset = 0;  // token offset inside that document
  o(0, 0) = 0;
  o(0, 1) = 0;
  for (int64_t s = 1; s <= n_samples; ++s) {
    int64_t remaining = seq_length + 1;
    while (remaining != 0) {
      if (pos >= ndoc_idx) throw std::runtime_error("build_sample_idx: ran out of documents");
      const int64_t doc_len = sz[di[pos]] - offset;
      remaining -= doc_len;
      if (remaining <= 0) {
        offset += remaining + doc_len - 1;  // last token is shared with the next sample
        remaining = 0;
      } else {
        ++pos;
        offset = 0;
      }
    }
    o(s, 0) = pos;
    o(s, 1) = offset;
  }
  return out;
}

// gather one sample (seq_len+1 tokens) into dst
template <typename TokT>
static void gather_sample(const TokT* tokens, const int64_t* doc_off, const int32_t* doc_idx,
                          const int64_t* sample_idx, int64_t s, int64_t seq1, int64_t* dst) {
  int64_t pos = sample_idx[2 * s], off = sample_idx[2 * s + 1];
  const int64_t pos_end = sample_idx[2 * (s + 1)], off_end = sample_idx[2 * (s + 1) + 1];
  int64_t n = 0;
  while (n < seq1) {
    const int64_t d = doc_idx[pos];
    const int64_t start = doc_off[d] + off;
    int64_t len = (pos == pos_end) ? (off_end - off + 1) : (doc_off[d + 1] - start);
    len = std::min(len, seq1 - n);
    for (int64_t i = 0; i < len; ++i) dst[n + i] = (int64_t)tokens[start + i];
    n += len;
    ++pos;
    off = 0;
  }
}

class TokenLoader {
 public:
  TokenLoader(uintptr_t tokens, int elem_bytes, py::array_t<int64_t, py::array::c_style | py::array::forcecast> doc_off,
              py::array_t<int32_t, py::array::c_style | py::array::forcecast> doc_idx,
              py::array_t<int64_t, py::array::c_style | py::array::forcecast> sample_idx,
              py::array_t<int64_t, py::array::c_style | py::array::forcecast> shuffle_idx, int64_t batch,
              int64_t seq_len, std::vector<uintptr_t> slots, int nthreads)
      : tokens_((const void*)tokens), elem_(elem_bytes), doc_off_(doc_off), doc_idx_(doc_idx),
        sample_idx_(sample_idx), shuffle_(shuffle_idx), batch_(batch), seq1_(seq_len + 1),
        slots_(slots), state_(slots.size(), kFree), owner_(slots.size(), -1) {
    if (elem_ != 2 && elem_ != 4 && elem_ != 8) throw std::invalid_argument("token width must be 2/4/8 bytes");
    if (slots_.empty()) throw std::invalid_argument("need at least one ring slot");
    n_batches_ = (int64_t)shuffle_.size() / batch_;
    nthreads_ = std::max(1, nthreads);
  }
  ~TokenLoader() { stop(); }

  int64_t num_batches() const { return n_batches_; }

  void start(int64_t first_batch) {
    stop();
    {
      std::lock_guard<std::mutex> g(mu_);
      stopping_ = false;
      next_fill_ = first_batch;
      next_get_ = first_batch;
      std::fill(state_.begin(), state_.end(), kFree);
      std::fill(owner_.begin(), owner_.end(), -1);
    }
    for (int i = 0; i < nthreads_; ++i) workers_.emplace_back([this] { run(); });
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stopping_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
    workers_.clear();
  }

  // blocks until the next batch is filled; returns (slot, batch number) or (-1, -1) at end
  std::pair<int, int64_t> acquire() {
    py::gil_scoped_release nogil;
    std::unique_lock<std::mutex> lk(mu_);
    const int64_t b = next_get_;
    if (b >= n_batches_) return {-1, -1};
    const int slot = (int)(b % (int64_t)slots_.size());
    cv_.wait(lk, [&] { return (state_[slot] == kReady && owner_[slot] == b) || stopping_; });
    if (stopping_) return {-1, -1};
    state_[slot] = kInUse;
    ++next_get_;
    return {slot, b};
  }

  void release(int slot) {
    {
      std::lock_guard<std::mutex> g(mu_);
      state_[slot] = kFree;
      owner_[slot] = -1;
    }
    cv_.notify_all();
  }

 private:
  enum { kFree = 0, kFilling = 1, kReady = 2, kInUse = 3 };

  void run() {
    for (;;) {
      int64_t b;
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          if (stopping_ || next_fill_ >= n_batches_) return true;
          const int s = (int)(next_fill_ % (int64_t)slots_.size());
          // only fill a slot once the consumer is within one ring of this batch
          return state_[s] == kFree && next_fill_ < next_get_ + (int64_t)slots_.size();
        });
        if (stopping_ || next_fill_ >= n_batches_) return;
        b = next_fill_++;
        slot = (int)(b % (int64_t)slots_.size());
        state_[slot] = kFilling;
        owner_[slot] = b;
      }
      fill(b, (int64_t*)slots_[slot]);
      {
        std::lock_guard<std::mutex> g(mu_);
        state_[slot] = kReady;
      }
      cv_.notify_all();
    }
  }

  void fill(int64_t b, int64_t* dst) {
    const int64_t* off = doc_off_.data();
    const int32_t* di = doc_idx_.data();
    const int64_t* si = sample_idx_.data();
    const int64_t* sh = shuffle_.data();
    for (int64_t i = 0; i < batch_; ++i) {
      const int64_t s = sh[b * batch_ + i];
      int64_t* row = dst + i * seq1_;
      if (elem_ == 2)
        gather_sample((const uint16_t*)tokens_, off, di, si, s, seq1_, row);
      else if (elem_ == 4)
        gather_sample((const int32_t*)tokens_, off, di, si, s, seq1_, row);
      else
        gather_sample((const int64_t*)tokens_, off, di, si, s, seq1_, row);
    }
  }

  const void* tokens_;
  int elem_;
  py::array_t<int64_t> doc_off_;
  py::array_t<int32_t> doc_idx_;
  py::array_t<int64_t> sample_idx_;
  py::array_t<int64_t> shuffle_;
  int64_t batch_, seq1_, n_batches_ = 0;
  std::vector<uintptr_t> slots_;
  std::vector<int> state_;
  std::vector<int64_t> owner_;
  int nthreads_ = 1;
  int64_t next_fill_ = 0, next_get_ = 0;
  bool stopping_ = true;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::thread> workers_;
};

// dst[i*row_bytes : (i+1)*row_bytes] = srcs[i]  (all rows the same size), multi-threaded
void stack_rows(std::vector<uintptr_t> srcs, int64_t row_bytes, uintptr_t dst, int nthreads) {
  py::gil_scoped_release nogil;
  const int64_t n = (int64_t)srcs.size();
  nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, n));
  auto work = [&](int t) {
    for (int64_t i = t; i < n; i += nthreads)
      std::memcpy((char*)dst + i * row_bytes, (const void*)srcs[i], (size_t)row_bytes);
  };
  if (nthreads == 1 || n * row_bytes < (1 << 20)) {
    for (int64_t i = 0; i < n; ++i) std::memcpy((char*)dst + i * row_bytes, (const void*)srcs[i], (size_t)row_bytes);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
}

}  // namespace pra_data

void pra_register_data(py::module& m) {
  using namespace pra_data;
  m.def("build_sample_idx", &build_sample_idx, py::arg("sizes"), py::arg("doc_idx"), py::arg("seq_length"),
        py::arg("num_epochs"), py::arg("tokens_per_epoch"));
  m.def("stack_rows", &stack_rows, py::arg("srcs"), py::arg("row_bytes"), py::arg("dst"), py::arg("nthreads") = 4);
  py::class_<TokenLoader>(m, "TokenLoader")
      .def(py::init<uintptr_t, int, py::array_t<int64_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int64_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int64_t, py::array::c_style | py::array::forcecast>, int64_t, int64_t,
                    std::vector<uintptr_t>, int>())
      .def("start", &TokenLoader::start, py::arg("first_batch") = 0)
      .def("stop", &TokenLoader::stop)
      .def("acquire", &TokenLoader::acquire)
      .def("release", &TokenLoader::release)
      .def("num_batches", &TokenLoader::num_batches);
}
