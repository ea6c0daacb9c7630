"""Native (C++) runtime pieces: static-graph scheduler (``_pra_runtime``).

Built in-tree by ``python -m paddle_ray_amd.native.build`` (g++, pybind11). A pure
Python implementation of the same plan is kept for verification (tests assert
native == python) and as the fallback when the extension is not built.
"""
import glob
import importlib.util
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_mod = None


def runtime():
    global _mod
    if _mod is None:
        c = sorted(glob.glob(os.path.join(_HERE, '_pra_runtime*.so')))
        if not c:
            return None
        spec = importlib.util.spec_from_file_location('paddle_ray_amd.native._pra_runtime', c[0])
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        _mod = m
    return _mod


def build_plan_py(ins, outs, required, persistable):
    n = len(ins)
    producer = {}
    for i in range(n):
        for v in outs[i]:
            producer[v] = i
    live = [False] * n
    stack = []
    for v in required:
        if v in producer and not live[producer[v]]:
            live[producer[v]] = True
            stack.append(producer[v])
    for i in range(n):
        if not outs[i] and not live[i]:
            live[i] = True
            stack.append(i)
    while stack:
        op = stack.pop()
        for v in ins[op]:
            p = producer.get(v)
            if p is not None and not live[p]:
                live[p] = True
                stack.append(p)
    import heapq
    succ = [[] for _ in range(n)]
    indeg = [0] * n
    last_barrier = -1
    for j in range(n):
        if not live[j]:
            continue
        deps = {producer[v] for v in ins[j] if v in producer and producer[v] != j and live[producer[v]]}
        if last_barrier >= 0:
            deps.add(last_barrier)
        if not outs[j]:
            deps |= {i for i in range(j) if live[i]}
            last_barrier = j
        for d in deps:
            succ[d].append(j)
            indeg[j] += 1
    ready = [i for i in range(n) if live[i] and indeg[i] == 0]
    heapq.heapify(ready)
    order, level, lvl = [], [], [0] * n
    while ready:
        op = heapq.heappop(ready)
        order.append(op)
        level.append(lvl[op])
        for s in succ[op]:
            lvl[s] = max(lvl[s], lvl[op] + 1)
            indeg[s] -= 1
            if indeg[s] == 0:
                heapq.heappush(ready, s)
    pruned = [i for i in range(n) if not live[i]]
    keep = set(persistable) | set(required)
    last = {}
    for p, op in enumerate(order):
        for v in ins[op]:
            last[v] = p
        for v in outs[op]:
            last.setdefault(v, p)
    free_after = [[] for _ in order]
    for v, p in last.items():
        if v not in keep:
            free_after[p].append(v)
    for f in free_after:
        f.sort()
    return order, free_after, level, pruned


def build_plan(ins, outs, required, persistable):
    rt = runtime()
    if rt is not None:
        return rt.build_plan(ins, outs, list(required), list(persistable))
    return build_plan_py(ins, outs, required, persistable)
