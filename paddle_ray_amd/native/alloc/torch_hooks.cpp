// PyTorch-ROCm integration of the native auto-growth allocator (auto_growth_allocator.cpp):
// builds a CUDAPluggableAllocator from the allocator's C entry points (passed in as addresses
// of the ctypes-loaded _pra_alloc_hip.so, so statistics read through ctypes see the same
// instance) and installs the graph-capture pool hooks that the ctypes-only pluggable path
// cannot set:
//   beginAllocateToPool(device, pool, filter): allocations on streams the filter accepts (the
//     streams being captured) go to the pool's private arena until endAllocateToPool;
//   releasePool(device, pool): the graph is gone; the arena is freed with its last block;
//   recordStream(ptr, stream): the block's free waits for that stream's work as well.
// Parity: the reference's CUDAGraph private memory pools (paddle/fluid/memory/allocation/
// allocator_facade.cc, PrepareMemoryPoolForCUDAGraph / RemoveMemoryPoolOfCUDAGraph).
#include <torch/extension.h>
#include <torch/csrc/cuda/CUDAPluggableAllocator.h>

#include <map>
#include <mutex>
#include <vector>

namespace {

typedef void* (*alloc_t)(size_t, int, hipStream_t);
typedef void (*free_t)(void*, size_t, int, hipStream_t);
typedef void* (*alloc_pool_t)(size_t, int, hipStream_t, uint64_t, uint64_t);
typedef void (*release_t)(int, uint64_t, uint64_t);
typedef void (*record_t)(void*, hipStream_t);

struct Active {
  c10::hip::MempoolId_t id;
  std::function<bool(hipStream_t)> filter;
};
std::mutex g_mu;
std::map<int, std::vector<Active>> g_active;  // pools being allocated into, per device
int64_t g_pool_allocs = 0;

bool install(uintptr_t a, uintptr_t f, uintptr_t ap, uintptr_t rel, uintptr_t rec) {
  const alloc_t A = reinterpret_cast<alloc_t>(a);
  const free_t F = reinterpret_cast<free_t>(f);
  const alloc_pool_t AP = reinterpret_cast<alloc_pool_t>(ap);
  const release_t R = reinterpret_cast<release_t>(rel);
  auto alloc = torch::cuda::CUDAPluggableAllocator::createCustomAllocator(
      [A, AP](size_t n, int d, hipStream_t s) -> void* {
        {
          std::lock_guard<std::mutex> g(g_mu);
          auto it = g_active.find(d);
          if (it != g_active.end())
            for (auto r = it->second.rbegin(); r != it->second.rend(); ++r)
              if (r->filter(s)) {
                ++g_pool_allocs;
                return AP(n, d, s, r->id.first, r->id.second);
              }
        }
        return A(n, d, s);
      },
      [F](void* p, size_t n, int d, hipStream_t s) { F(p, n, d, s); });
  auto* pa = dynamic_cast<torch::cuda::CUDAPluggableAllocator::CUDAPluggableAllocator*>(alloc.get());
  if (!pa) return false;
  pa->set_begin_allocate_to_pool(
      [](int d, c10::hip::MempoolId_t id, std::function<bool(hipStream_t)> filter) {
        std::lock_guard<std::mutex> g(g_mu);
        g_active[d].push_back(Active{id, std::move(filter)});
      });
  pa->set_end_allocate_to_pool_fn([](int d, c10::hip::MempoolId_t id) {
    std::lock_guard<std::mutex> g(g_mu);
    auto& v = g_active[d];
    for (auto it = v.begin(); it != v.end(); ++it)
      if (it->id == id) {
        v.erase(it);
        break;
      }
  });
  pa->set_release_pool([R](int d, c10::hip::MempoolId_t id) { R(d, id.first, id.second); });
  if (rec) {
    const record_t RS = reinterpret_cast<record_t>(rec);
    pa->set_record_stream_fn([RS](void* p, hipStream_t s) { RS(p, s); });
  }
  torch::cuda::CUDAPluggableAllocator::changeCurrentAllocator(alloc);
  return true;
}

int64_t pool_allocs() {
  std::lock_guard<std::mutex> g(g_mu);
  return g_pool_allocs;
}

}  // namespace

PYBIND11_MODULE(_pra_alloc_torch, m) {
  m.def("install", &install, "make the native allocator PyTorch's device allocator (with graph pools)");
  m.def("pool_allocs", &pool_allocs, "allocations served from graph-capture pools so far");
}
