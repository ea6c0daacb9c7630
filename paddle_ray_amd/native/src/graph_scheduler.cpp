// Native static-graph scheduler for paddle_ray_amd.static.Executor.
//
// Parity: paddle/fluid/framework/new_executor/interpretercore.cc +
// interpreter/dependency_builder.cc (op dependency analysis, instruction
// scheduling) and garbage_collector/ (free a variable after its last use).
//
// Input : ops as (input var ids, output var ids), the set of fetch/required var
//         ids and persistable var ids.
// Output: an execution plan = ops pruned to those that (transitively) feed a
//         required var, in a dependency-respecting order (Kahn, stable by
//         program order), plus for every step the var ids whose LAST use is that
//         step (the executor drops them -> HBM returns to the caching allocator
//         early), plus a "level" per op (ops of equal level are independent and
//         could be dispatched on separate HIP streams).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <queue>
#include <stdexcept>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace py = pybind11;

struct Plan {
  std::vector<int> order;                   // op indices to execute
  std::vector<std::vector<int>> free_after;  // per position in `order`: var ids to release
  std::vector<int> level;                   // per position in `order`
  std::vector<int> pruned;                  // op indices removed as dead code
};

static Plan build_plan(const std::vector<std::vector<int>>& ins, const std::vector<std::vector<int>>& outs,
                       const std::vector<int>& required, const std::vector<int>& persistable) {
  const int n = (int)ins.size();
  if ((int)outs.size() != n) throw std::invalid_argument("ins/outs size mismatch");
  // producer of each var (last writer wins, like sequential program semantics)
  std::unordered_map<int, int> producer;
  for (int i = 0; i < n; ++i)
    for (int v : outs[i]) producer[v] = i;
  // backward liveness: keep ops that produce a required var (transitively)
  std::vector<char> live(n, 0);
  std::vector<int> stack;
  std::unordered_set<int> need(required.begin(), required.end());
  for (int v : required) {
    auto it = producer.find(v);
    if (it != producer.end() && !live[it->second]) { live[it->second] = 1; stack.push_back(it->second); }
  }
  // ops with no outputs (side effects: optimizer/backward markers) are always live
  for (int i = 0; i < n; ++i)
    if (outs[i].empty() && !live[i]) { live[i] = 1; stack.push_back(i); }
  while (!stack.empty()) {
    int op = stack.back();
    stack.pop_back();
    for (int v : ins[op]) {
      auto it = producer.find(v);
      if (it != producer.end() && it->second < op + 1 && !live[it->second]) {
        live[it->second] = 1;
        stack.push_back(it->second);
      } else if (it != producer.end() && !live[it->second]) {
        live[it->second] = 1;
        stack.push_back(it->second);
      }
    }
  }
  // dependency graph among live ops: op j depends on producer(v) for v in ins[j],
  // and side-effect ops (no outputs) are ordered after every earlier live op
  std::vector<std::vector<int>> succ(n);
  std::vector<int> indeg(n, 0);
  int last_barrier = -1;
  for (int j = 0; j < n; ++j) {
    if (!live[j]) continue;
    std::unordered_set<int> deps;
    for (int v : ins[j]) {
      auto it = producer.find(v);
      if (it != producer.end() && it->second != j && live[it->second]) deps.insert(it->second);
    }
    if (last_barrier >= 0) deps.insert(last_barrier);
    if (outs[j].empty()) {
      for (int i = 0; i < j; ++i)
        if (live[i]) deps.insert(i);
      last_barrier = j;
    }
    for (int d : deps) { succ[d].push_back(j); ++indeg[j]; }
  }
  // Kahn with a min-heap on program index (stable: preserves program order when free)
  Plan plan;
  std::priority_queue<int, std::vector<int>, std::greater<int>> ready;
  std::vector<int> lvl(n, 0);
  for (int i = 0; i < n; ++i)
    if (live[i] && indeg[i] == 0) ready.push(i);
  while (!ready.empty()) {
    int op = ready.top();
    ready.pop();
    plan.order.push_back(op);
    plan.level.push_back(lvl[op]);
    for (int s : succ[op]) {
      lvl[s] = std::max(lvl[s], lvl[op] + 1);
      if (--indeg[s] == 0) ready.push(s);
    }
  }
  int nlive = 0;
  for (int i = 0; i < n; ++i) nlive += live[i];
  if ((int)plan.order.size() != nlive) throw std::runtime_error("cycle in program graph");
  for (int i = 0; i < n; ++i)
    if (!live[i]) plan.pruned.push_back(i);
  // last use of each non-persistable, non-required var
  std::unordered_set<int> keep(persistable.begin(), persistable.end());
  keep.insert(required.begin(), required.end());
  std::unordered_map<int, int> last_use;
  for (int p = 0; p < (int)plan.order.size(); ++p) {
    int op = plan.order[p];
    for (int v : ins[op]) last_use[v] = p;
    for (int v : outs[op])
      if (!last_use.count(v)) last_use[v] = p;  // produced but never read
  }
  plan.free_after.assign(plan.order.size(), {});
  for (auto& kv : last_use)
    if (!keep.count(kv.first)) plan.free_after[kv.second].push_back(kv.first);
  for (auto& f : plan.free_after) std::sort(f.begin(), f.end());
  return plan;
}

void pra_register_data(py::module& m);  // data_ring.cpp

PYBIND11_MODULE(_pra_runtime, m) {
  m.doc() = "paddle_ray_amd native runtime: static-graph scheduler + data pipeline";
  pra_register_data(m);
  m.def("build_plan",
        [](const std::vector<std::vector<int>>& ins, const std::vector<std::vector<int>>& outs,
           const std::vector<int>& required, const std::vector<int>& persistable) {
          Plan p = build_plan(ins, outs, required, persistable);
          return py::make_tuple(p.order, p.free_after, p.level, p.pruned);
        },
        py::arg("ins"), py::arg("outs"), py::arg("required"), py::arg("persistable"));
}
