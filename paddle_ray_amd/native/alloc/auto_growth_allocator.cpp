// Auto-growth best-fit device allocator with per-stream free lists.
//
// Parity: paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc (chunks grown on
// demand, best-fit block search, block splitting and neighbour coalescing, free chunks
// released on demand) and stream_safe_cuda_allocator.cc (a block freed on stream S is reused
// by stream S without synchronisation; another stream only takes it after the event
// recorded at free time completed). Plugged into PyTorch-ROCm through
// torch.cuda.memory.CUDAPluggableAllocator (pra_alloc / pra_free) so every framework tensor
// comes from it when enabled; statistics feed paddle.device.cuda.memory_* .
//
// Graph-capture pools: while a HIP graph is being captured, allocations on the capturing
// streams come from a private arena keyed by the graph's pool id (the reference's
// CUDAGraph-private memory pools; PyTorch's beginAllocateToPool / endAllocateToPool /
// releasePool): blocks the graph uses are never handed to eager code, frees inside the capture
// are reused in stream order within the same arena, and the arena's memory returns to the device
// when the pool is released and its last block freed. No events are recorded for pool blocks (a
// capturing stream cannot be queried). torch_hooks.cpp wires these entry points into PyTorch.
//
// Built twice: with hipcc against the HIP runtime (the real allocator), and with
// -DPRA_ALLOC_HOST against malloc so the block bookkeeping is unit-tested on the CPU.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <unordered_map>
#include <vector>

#ifdef PRA_ALLOC_HOST
// Host build: an "event" is a flag that is pending until the test completes it
// (pra_alloc_host_complete_events), or done at once unless pending mode is on.
struct HostEvent {
  bool done;
};
typedef void* stream_t;
typedef HostEvent* event_t;
static bool g_host_pending = false;
static std::vector<HostEvent*> g_host_events;
static int backend_malloc(void** p, size_t n) {
  *p = std::aligned_alloc(256, n);
  return *p ? 0 : 1;
}
static void backend_free(void* p) { std::free(p); }
static void backend_set_device(int) {}
static event_t event_record(stream_t) {
  HostEvent* e = new HostEvent{!g_host_pending};
  g_host_events.push_back(e);
  return e;
}
static bool event_done(event_t e) { return e == nullptr || e->done; }
static void event_destroy(event_t) {}
static void device_sync() {
  for (HostEvent* e : g_host_events) e->done = true;
}
#else
#include <hip/hip_runtime.h>
typedef hipStream_t stream_t;
typedef hipEvent_t event_t;
// hipMalloc / hipFree / hipDeviceSynchronize while a stream capture is open on this thread:
// relaxed capture mode for the call (as PyTorch's caching allocator does), else the runtime
// invalidates the capture ("potentially unsafe API" under the default global mode)
struct RelaxedCapture {
  hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
  RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
  ~RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&m); }
};
static int backend_malloc(void** p, size_t n) {
  RelaxedCapture g;
  return hipMalloc(p, n) == hipSuccess ? 0 : 1;
}
static void backend_free(void* p) {
  RelaxedCapture g;
  (void)hipFree(p);
}
static void backend_set_device(int d) { (void)hipSetDevice(d); }
static event_t event_record(stream_t s) {
  event_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
  (void)hipEventRecord(e, s);
  return e;
}
static bool event_done(event_t e) { return e == nullptr || hipEventQuery(e) == hipSuccess; }
static void event_destroy(event_t e) {
  if (e) (void)hipEventDestroy(e);
}
static void device_sync() {
  RelaxedCapture g;
  (void)hipDeviceSynchronize();
}
#endif

namespace {

constexpr size_t kAlign = 256;
constexpr size_t kMinSplit = 512;  // remainders smaller than this stay with the block

struct Chunk;
struct Block {
  char* ptr;
  size_t size;
  bool free;
  Chunk* chunk;
  Block* prev;  // address-ordered neighbours inside the chunk
  Block* next;
  stream_t stream;  // stream of the last user
  event_t event;    // recorded on `stream` when freed (cross-stream reuse gate)
  std::vector<stream_t> rec;  // other streams that used the block (record_stream)
};

struct Chunk {
  char* base;
  size_t size;
  Block* head;
};

struct Stats {
  int64_t allocated = 0, reserved = 0, peak_allocated = 0, peak_reserved = 0;
  int64_t n_alloc = 0, n_free = 0, n_chunks = 0, n_backend_alloc = 0, n_backend_free = 0;
};

struct DeviceAllocator {
  std::mutex mu;
  size_t growth = size_t(64) << 20;  // minimum chunk size
  bool pool = false;                 // a graph-capture arena: no events, stream-order reuse only
  bool released = false;             // pool released while blocks were still live
  // Events only matter once a second stream allocates: until then every block is reused in
  // stream order and frees record nothing. When a second stream first shows up the device
  // is synchronised once (all earlier, event-less frees are then complete).
  stream_t first_stream = nullptr;
  bool seen_stream = false, multi_stream = false;
  std::vector<event_t> event_pool;
  // free blocks per stream, ordered by (size, address) -> best fit = lower_bound
  std::map<stream_t, std::set<std::pair<size_t, Block*>>> free_sets;
  std::unordered_map<void*, Block*> live;
  std::vector<Chunk*> chunks;
  // freed blocks that record_stream tied to other streams: they stay allocated until the
  // events recorded on those streams at free time complete (PyTorch's recordStream contract)
  std::vector<std::pair<Block*, std::vector<event_t>>> deferred;
  Stats st;

  static size_t round(size_t n) { return ((n ? n : 1) + kAlign - 1) / kAlign * kAlign; }

  void insert_free(Block* b) { free_sets[b->stream].insert({b->size, b}); }
  void erase_free(Block* b) {
    auto it = free_sets.find(b->stream);
    if (it != free_sets.end()) it->second.erase({b->size, b});
  }

  void note_stream(stream_t s) {
    if (pool) return;
    if (!seen_stream) {
      seen_stream = true;
      first_stream = s;
    } else if (!multi_stream && s != first_stream) {
      device_sync();
      multi_stream = true;
    }
  }
  event_t new_event(stream_t s) {
    if (!multi_stream || pool) return nullptr;
#ifdef PRA_ALLOC_HOST
    return event_record(s);
#else
    if (event_pool.empty()) return event_record(s);
    event_t e = event_pool.back();
    event_pool.pop_back();
    (void)hipEventRecord(e, s);
    return e;
#endif
  }
  void drop_event(Block* b) {
    if (b->event) {
      event_pool.push_back(b->event);
      b->event = nullptr;
    }
  }

  Block* take(Block* b, size_t n, stream_t s) {
    erase_free(b);
    // a block taken from its own stream's list may still be in use by work queued on that
    // stream before its free: the split remainder keeps a gate of its own, recorded on that
    // stream now (it completes after that work), so another stream cannot take it early
    const bool pending = !event_done(b->event);
    const stream_t old_stream = b->stream;
    drop_event(b);
    if (b->size - n >= kMinSplit) {  // split: remainder stays free on the block's stream
      Block* r = new Block{b->ptr + n, b->size - n, true, b->chunk, b, b->next, b->stream,
                           pending ? new_event(old_stream) : nullptr};
      if (b->next) b->next->prev = r;
      b->next = r;
      b->size = n;
      insert_free(r);
    }
    b->free = false;
    b->stream = s;
    live[b->ptr] = b;
    st.allocated += (int64_t)b->size;
    st.peak_allocated = std::max(st.peak_allocated, st.allocated);
    st.n_alloc++;
    return b;
  }

  Block* find(size_t n, stream_t s) {
    auto it = free_sets.find(s);
    if (it != free_sets.end()) {
      auto f = it->second.lower_bound({n, nullptr});
      if (f != it->second.end()) return f->second;
    }
    // another stream's block, once the work queued before its free has completed
    Block* best = nullptr;
    for (auto& kv : free_sets) {
      if (kv.first == s) continue;
      for (auto f = kv.second.lower_bound({n, nullptr}); f != kv.second.end(); ++f) {
        if (event_done(f->second->event)) {
          if (!best || f->second->size < best->size) best = f->second;
          break;
        }
      }
    }
    return best;
  }

  bool grow(size_t n) {
    size_t csz = std::max(n, growth);
    csz = (csz + (size_t(2) << 20) - 1) / (size_t(2) << 20) * (size_t(2) << 20);
    void* p = nullptr;
    if (backend_malloc(&p, csz) != 0) return false;
    Chunk* c = new Chunk{(char*)p, csz, nullptr};
    Block* b = new Block{(char*)p, csz, true, c, nullptr, nullptr, nullptr, nullptr};
    c->head = b;
    chunks.push_back(c);
    insert_free(b);
    st.reserved += (int64_t)csz;
    st.peak_reserved = std::max(st.peak_reserved, st.reserved);
    st.n_chunks++;
    st.n_backend_alloc++;
    return true;
  }

  // release chunks that are one free block; returns bytes released
  size_t release_free_chunks() {
    size_t freed = 0;
    std::vector<Chunk*> keep;
    for (Chunk* c : chunks) {
      Block* b = c->head;
      if (b->free && b->next == nullptr && b->size == c->size && event_done(b->event)) {
        erase_free(b);
        drop_event(b);
        backend_free(c->base);
        st.reserved -= (int64_t)c->size;
        st.n_chunks--;
        st.n_backend_free++;
        freed += c->size;
        delete b;
        delete c;
      } else {
        keep.push_back(c);
      }
    }
    chunks.swap(keep);
    return freed;
  }

  void* alloc(size_t size, stream_t s) {
    std::lock_guard<std::mutex> g(mu);
    note_stream(s);
    if (!deferred.empty()) process_deferred();
    const size_t n = round(size);
    Block* b = find(n, s);
    if (!b) {
      if (!grow(n)) {  // out of memory: wait for pending frees, drop free chunks, retry
        device_sync();
        process_deferred();
        release_free_chunks();
        if (!grow(n)) return nullptr;
      }
      b = find(n, s);
      if (!b) return nullptr;
    }
    return take(b, n, s)->ptr;
  }

  // another stream uses a live block: its free must wait for that stream's work too
  bool record_stream(void* p, stream_t s2) {
    std::lock_guard<std::mutex> g(mu);
    auto it = live.find(p);
    if (it == live.end()) return false;
    Block* b = it->second;
    if (pool || s2 == b->stream) return true;
    note_stream(s2);
    if (std::find(b->rec.begin(), b->rec.end(), s2) == b->rec.end()) b->rec.push_back(s2);
    return true;
  }

  void process_deferred() {
    std::vector<std::pair<Block*, std::vector<event_t>>> keep;
    for (auto& d : deferred) {
      bool done = true;
      for (event_t e : d.second) done = done && event_done(e);
      if (!done) {
        keep.push_back(std::move(d));
        continue;
      }
      for (event_t e : d.second)
        if (e) event_pool.push_back(e);
      // a fresh gate on the freeing stream: neighbours freed there since then may merge in,
      // and the merged block must wait for their work too
      Block* b = d.first;
      drop_event(b);
      release(b, b->stream, new_event(b->stream));
    }
    deferred.swap(keep);
  }

  void free_(void* p, stream_t s) {
    std::lock_guard<std::mutex> g(mu);
    auto it = live.find(p);
    if (it == live.end()) return;
    Block* b = it->second;
    live.erase(it);
    st.n_free++;
    if (!b->rec.empty()) {
      std::vector<event_t> evs;
      for (stream_t r : b->rec)
        if (r != s) evs.push_back(new_event(r));
      b->rec.clear();
      b->stream = s;
      b->event = new_event(s);
      deferred.push_back({b, std::move(evs)});
      return;
    }
    release(b, s, new_event(s));
  }

  // a freed block (no other stream still using it) joins the free lists of stream s
  void release(Block* b, stream_t s, event_t ev) {
    st.allocated -= (int64_t)b->size;
    b->free = true;
    b->stream = s;
    b->event = ev;
    // coalesce with free neighbours freed on the same stream, or whose pending work is done
    // (their event completed: any stream may take them, so the merged block can be s's)
    auto mergeable = [&](Block* o) {
      return o && o->free && (o->stream == s || event_done(o->event));
    };
    if (mergeable(b->next)) {
      Block* n = b->next;
      erase_free(n);
      drop_event(n);
      b->size += n->size;
      b->next = n->next;
      if (n->next) n->next->prev = b;
      delete n;
    }
    if (mergeable(b->prev)) {
      Block* pr = b->prev;
      erase_free(pr);
      drop_event(pr);
      pr->size += b->size;
      pr->next = b->next;
      if (b->next) b->next->prev = pr;
      pr->event = b->event;  // the merged block is gated by this free's event
      pr->stream = s;
      b->event = nullptr;
      delete b;
      b = pr;
    }
    insert_free(b);
  }

  size_t live_count() const { return live.size(); }

  // bookkeeping invariant check (tests): blocks tile every chunk exactly, free sets agree
  bool check() {
    std::lock_guard<std::mutex> g(mu);
    size_t nfree = 0;
    for (auto& kv : free_sets) nfree += kv.second.size();
    size_t seen_free = 0;
    int64_t used = 0, reserved = 0;
    for (Chunk* c : chunks) {
      char* expect = c->base;
      for (Block* b = c->head; b; b = b->next) {
        if (b->ptr != expect || b->chunk != c) return false;
        if (b->next && b->next->prev != b) return false;
        expect += b->size;
        if (b->free) {
          seen_free++;
          if (!free_sets[b->stream].count({b->size, b})) return false;
        } else {
          used += (int64_t)b->size;
        }
      }
      if (expect != c->base + c->size) return false;
      reserved += (int64_t)c->size;
    }
    return seen_free == nfree && used == st.allocated && reserved == st.reserved;
  }
};

std::mutex g_mu;
std::map<int, DeviceAllocator*> g_dev;
// graph-capture arenas per (device, pool id), and which arena owns each live pointer
typedef std::pair<uint64_t, uint64_t> PoolId;
std::map<std::pair<int, PoolId>, DeviceAllocator*> g_pools;
std::mutex g_own_mu;
std::unordered_map<void*, DeviceAllocator*> g_owner;

DeviceAllocator* dev(int d) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_dev.find(d);
  if (it != g_dev.end()) return it->second;
  DeviceAllocator* a = new DeviceAllocator();
  if (const char* e = std::getenv("PRA_ALLOC_CHUNK_MB")) a->growth = size_t(std::atoll(e)) << 20;
  g_dev[d] = a;
  return a;
}

DeviceAllocator* pool_of(int d, PoolId id, bool create) {
  std::lock_guard<std::mutex> g(g_mu);
  auto key = std::make_pair(d, id);
  auto it = g_pools.find(key);
  if (it != g_pools.end()) return it->second;
  if (!create) return nullptr;
  DeviceAllocator* a = new DeviceAllocator();
  a->pool = true;
  a->growth = size_t(64) << 20;  // arenas grow like the device arena (64 MB chunks)
  g_pools[key] = a;
  return a;
}

// a released pool whose last block went away: return its memory to the device
void maybe_drop_pool(int d, DeviceAllocator* a) {
  bool drop = false;
  {
    std::lock_guard<std::mutex> g(a->mu);
    drop = a->released && a->live_count() == 0;
  }
  if (!drop) return;
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (auto it = g_pools.begin(); it != g_pools.end(); ++it)
      if (it->second == a && it->first.first == d) {
        g_pools.erase(it);
        break;
      }
  }
  {
    std::lock_guard<std::mutex> g(a->mu);
    a->release_free_chunks();
  }
  delete a;
}

}  // namespace

extern "C" {
// CUDAPluggableAllocator entry points
void* pra_alloc(size_t size, int device, stream_t stream) {
  backend_set_device(device);
  return dev(device)->alloc(size, stream);
}
void pra_free(void* ptr, size_t size, int device, stream_t stream) {
  (void)size;
  DeviceAllocator* owner = nullptr;
  {
    std::lock_guard<std::mutex> g(g_own_mu);
    auto it = g_owner.find(ptr);
    if (it != g_owner.end()) {
      owner = it->second;
      g_owner.erase(it);
    }
  }
  if (owner) {
    owner->free_(ptr, stream);
    maybe_drop_pool(device, owner);
    return;
  }
  dev(device)->free_(ptr, stream);
}
// PyTorch recordStream: the block at ptr is also used by stream s (device arenas only; graph
// pools reuse in capture order)
void pra_record_stream(void* ptr, stream_t stream) {
  {
    std::lock_guard<std::mutex> g(g_own_mu);
    if (g_owner.count(ptr)) return;
  }
  std::vector<DeviceAllocator*> devs;
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (auto& kv : g_dev) devs.push_back(kv.second);
  }
  for (DeviceAllocator* a : devs)
    if (a->record_stream(ptr, stream)) return;
}
// graph-capture arenas (pool id = PyTorch's MempoolId_t pair)
void* pra_alloc_pool(size_t size, int device, stream_t stream, uint64_t id0, uint64_t id1) {
  backend_set_device(device);
  DeviceAllocator* a = pool_of(device, PoolId(id0, id1), true);
  void* p = a->alloc(size, stream);
  if (p) {
    std::lock_guard<std::mutex> g(g_own_mu);
    g_owner[p] = a;
  }
  return p;
}
// the graph (and every private-pool user) is gone: free the arena once its blocks are
void pra_pool_release(int device, uint64_t id0, uint64_t id1) {
  DeviceAllocator* a = pool_of(device, PoolId(id0, id1), false);
  if (!a) return;
  {
    std::lock_guard<std::mutex> g(a->mu);
    a->released = true;
  }
  maybe_drop_pool(device, a);
}
// reserved / allocated bytes and arena count of the live pools of a device
void pra_pool_stats(int device, int64_t* out) {
  std::lock_guard<std::mutex> g(g_mu);
  int64_t res = 0, used = 0, n = 0;
  for (auto& kv : g_pools)
    if (kv.first.first == device) {
      std::lock_guard<std::mutex> g2(kv.second->mu);
      res += kv.second->st.reserved;
      used += kv.second->st.allocated;
      n++;
    }
  out[0] = used;
  out[1] = res;
  out[2] = n;
}
int pra_pool_check(int device, uint64_t id0, uint64_t id1) {
  DeviceAllocator* a = pool_of(device, PoolId(id0, id1), false);
  return a ? (a->check() ? 1 : 0) : -1;
}
// stats: allocated, reserved, peak_allocated, peak_reserved, n_alloc, n_free, n_chunks,
// n_backend_alloc, n_backend_free
void pra_alloc_stats(int device, int64_t* out) {
  DeviceAllocator* a = dev(device);
  std::lock_guard<std::mutex> g(a->mu);
  const Stats& s = a->st;
  int64_t v[9] = {s.allocated, s.reserved, s.peak_allocated, s.peak_reserved, s.n_alloc,
                  s.n_free, s.n_chunks, s.n_backend_alloc, s.n_backend_free};
  for (int i = 0; i < 9; ++i) out[i] = v[i];
}
void pra_alloc_reset_peak(int device) {
  DeviceAllocator* a = dev(device);
  std::lock_guard<std::mutex> g(a->mu);
  a->st.peak_allocated = a->st.allocated;
  a->st.peak_reserved = a->st.reserved;
}
int64_t pra_alloc_empty_cache(int device) {
  DeviceAllocator* a = dev(device);
  std::lock_guard<std::mutex> g(a->mu);
  return (int64_t)a->release_free_chunks();
}
void pra_alloc_set_growth(int device, int64_t bytes) {
  DeviceAllocator* a = dev(device);
  std::lock_guard<std::mutex> g(a->mu);
  a->growth = (size_t)bytes;
}
int pra_alloc_check(int device) { return dev(device)->check() ? 1 : 0; }
#ifdef PRA_ALLOC_HOST
// host-build test hooks: events recorded from now on stay pending until completed
void pra_alloc_host_set_pending(int on) { g_host_pending = on != 0; }
void pra_alloc_host_complete_events() {
  for (HostEvent* e : g_host_events) e->done = true;
}
#endif
}
