"""Topology-aware GPU-set selection for multi-GPU requests (GetPreferredAllocation).

Reference: go-gpuallocator ``besteffort_policy.go`` — ``Allocate`` (:34-89) picks the
highest-scoring *partition* of all available GPUs into sets of ``size`` (padded with
``None``) among partitions that have an unpadded set containing every ``required`` GPU,
then returns the best-scoring such set; pair scores (:298-356) are 100 x NVLink count or
a PCIe-distance level (cross-CPU 10 ... same-board 60); set score = sum of pair scores
(:360-380). The reference enumerates partitions recursively (exponential).

MI355X version:
* pair score from the KFD io_links: xGMI = 100 per direct link (an 8-GPU MI355X UBB
  connects every pair with one link, so all pairs tie at 100), PCIe = 20 on the same NUMA
  node, 10 across; plus 1 for the same NUMA node so ties break toward CPU locality;
* the same objective is solved exactly with a memoised search over bitmasks:
  best(mask) = max over sets S containing the lowest remaining GPU of
  score(S) + best(mask \\ S). For <= 16 GPUs this is milliseconds, and it returns the
  reference's answer (tests/test_topology.py checks it against a brute-force port of the
  reference's recursion).
"""
from functools import lru_cache
from itertools import combinations

IOLINK_PCIE = 2
IOLINK_XGMI = 11


def pair_score(a, b):
    """Link score between two GpuDevice (0 for padding/self)."""
    if a is None or b is None or a is b:
        return 0
    score = 0
    links = a.links.get(b.index, [])
    for ltype, _w in links:
        if ltype == IOLINK_XGMI:
            score += 100
        elif ltype == IOLINK_PCIE:
            score += 20 if (a.numa_node == b.numa_node and a.numa_node >= 0) else 10
    if not links:
        score += 20 if (a.numa_node == b.numa_node and a.numa_node >= 0) else 10
    if a.numa_node == b.numa_node and a.numa_node >= 0:
        score += 1
    return score


def set_score(devs):
    return sum(pair_score(a, b) for a, b in combinations(devs, 2))


def best_effort(available, required, size):
    """Returns the preferred list of GpuDevice (len == size) or [] when impossible."""
    if size <= 0 or len(available) < size or len(required) > size:
        return []
    avail = list(available)
    if any(r not in avail for r in required):
        return []
    n = len(avail)
    if size == 1:
        if required:
            return [required[0]]
        return [avail[0]]
    pad = (-n) % size
    items = avail + [None] * pad
    N = len(items)
    req_idx = frozenset(avail.index(r) for r in required)
    pair = [[pair_score(items[i], items[j]) for j in range(N)] for i in range(N)]

    def sscore(idxs):
        return sum(pair[i][j] for i, j in combinations(idxs, 2))

    def npad(idxs):
        return sum(1 for i in idxs if i >= n)

    @lru_cache(maxsize=None)
    def best(mask):
        """(score, partition) of the best partition of ``mask`` into padded sets."""
        if mask == 0:
            return 0, ()
        idx = [i for i in range(N) if mask >> i & 1]
        first, rest = idx[0], idx[1:]
        top = None
        for comb in combinations(rest, size - 1):
            s = (first,) + comb
            p = npad(s)
            if p not in (0, pad):  # reference: only sets with no or all padding
                continue
            m = mask
            for i in s:
                m &= ~(1 << i)
            sub, parts = best(m)
            cand = (sscore(s) + sub, (s,) + parts)
            if top is None or cand[0] > top[0]:
                top = cand
        return top if top else (float("-inf"), ())

    full = (1 << N) - 1
    best_total, best_sets = None, None
    if req_idx:
        # The set holding the required GPUs is unpadded and contains all of them.
        others = [i for i in range(n) if i not in req_idx]
        for comb in combinations(others, size - len(req_idx)):
            s = tuple(sorted(req_idx | set(comb)))
            m = full
            for i in s:
                m &= ~(1 << i)
            sub, parts = best(m)
            total = sscore(s) + sub
            if best_total is None or total > best_total:
                best_total, best_sets = total, (s,)
        chosen = best_sets[0] if best_sets else None
    else:
        _, parts = best(full)
        cands = [s for s in parts if npad(s) == 0]
        chosen = max(cands, key=sscore) if cands else None
    if chosen is None:
        return []
    return [items[i] for i in chosen]


PLACEMENT_SPREAD, PLACEMENT_BINPACK = "spread", "binpack"
PLACEMENTS = (PLACEMENT_SPREAD, PLACEMENT_BINPACK)


def _placement_key(placement, free, order):
    """Sort key of a physical GPU for ``placement``: spread prefers the GPU with the most
    free vGPUs (tenants land on idle GPUs first, so each keeps its spatial CU slice and
    the node's 8 GPUs fill evenly); binpack the one with the fewest (whole GPUs stay free
    for large jobs). Ties keep the kubelet's order."""
    return (-free if placement == PLACEMENT_SPREAD else free, order)


def allocate_vdevices(vdevices, available_ids, must_include_ids, size, placement=PLACEMENT_SPREAD):
    """GetPreferredAllocation for vGPU ids (reference ``server.go:271-326``).

    Maps the available vGPU ids onto their physical GPUs and picks ``size`` distinct GPUs:
    the best-effort topology policy decides first (for multi-GPU requests), and among
    GPU sets of equal topology score the ``placement`` policy decides, with the number of
    free vGPUs per GPU taken from the kubelet's own ``available`` list. Each chosen GPU is
    mapped back to one of its available vGPUs - a must-include vGPU when there is one (the
    reference always takes the first available vGPU of the GPU, ignoring must-include).

    The reference's fallback (the first ``size`` available ids, ``server.go:305-310``) may
    return two vGPUs of one GPU while other GPUs have free slots. Here two vGPUs of one GPU
    are only returned when fewer than ``size`` distinct GPUs have a free vGPU (and then
    ``Allocate`` decides, see ``--duplicate-vgpus``), and a 1-vGPU request goes to the GPU
    the placement policy picks instead of the first available one.
    """
    by_id = {v.id: v for v in vdevices}
    avail = [by_id[i] for i in available_ids if i in by_id]
    must = [by_id[i] for i in must_include_ids if i in by_id]
    free, order, phys = {}, {}, []
    for v in avail:
        free[v.uuid] = free.get(v.uuid, 0) + 1
        if v.uuid not in order:
            order[v.uuid] = len(order)
            phys.append(v.dev)
    req_phys, rseen = [], set()
    for v in must:
        if v.uuid not in rseen:
            rseen.add(v.uuid)
            p = next((p for p in phys if p.uuid == v.uuid), None)
            if p is not None:
                req_phys.append(p)
    key = lambda p: _placement_key(placement, free.get(p.uuid, 0), order.get(p.uuid, 0))  # noqa: E731
    chosen = []
    if len(req_phys) == len(rseen) == len(must) and len(phys) >= size:
        if size == 1:
            chosen = req_phys[:1] or [min(phys, key=key)]
        else:
            best = best_effort(phys, req_phys, size)
            if best:
                chosen = _placement_among_ties(phys, req_phys, size, set_score(best), key) or best
    if chosen:
        out = []
        for p in chosen:
            pick = next((v for v in must if v.uuid == p.uuid), None) or next(v for v in avail if v.uuid == p.uuid)
            out.append(pick.id)
        return out
    # Fewer distinct GPUs than requested (or must-includes that are not available): every
    # must-include, then one vGPU of each other GPU in placement order, and only then
    # second vGPUs of GPUs already chosen.
    out = [v.id for v in must]
    used = {by_id[i].uuid for i in out}
    for p in sorted(phys, key=key):
        if len(out) >= size:
            break
        if p.uuid not in used:
            out.append(next(v.id for v in avail if v.uuid == p.uuid))
            used.add(p.uuid)
    for v in avail:
        if len(out) >= size:
            break
        if v.id not in out:
            out.append(v.id)
    return out[:size]


def _placement_among_ties(phys, required, size, score, key, limit=20000):
    """Among the GPU sets of ``size`` holding ``required`` whose topology score equals
    ``score`` (the best-effort answer's), the one the placement key prefers (summed over
    the set). Bounded enumeration: None when there are too many sets to look at."""
    from math import comb
    others = [p for p in phys if p not in required]
    k = size - len(required)
    if k < 0 or comb(len(others), k) > limit:
        return None
    best, best_key = None, None
    for c in combinations(sorted(others, key=key), k):
        s = list(required) + list(c)
        if set_score(s) != score:
            continue
        kk = tuple(sum(x) for x in zip(*(key(p) for p in s)))
        if best is None or kk < best_key:
            best, best_key = s, kk
    return best
