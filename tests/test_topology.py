"""Best-effort GPU-set policy vs an exhaustive enumeration of the reference's objective
(go-gpuallocator besteffort_policy.go:34-89: best partition into padded sets of `size`,
constrained to contain an unpadded set holding every required GPU)."""
import itertools
import random

from hypothesis import given, settings, strategies as st

from amdvgpu.parallel.topology import IOLINK_PCIE, IOLINK_XGMI, allocate_vdevices, best_effort, pair_score, set_score
from amdvgpu.plugin.devices import FakeBackend, GpuDevice
from amdvgpu.plugin.vdevice import device_to_vdevices


def partitions(items, size):
    if not items:
        yield []
        return
    first, rest = items[0], items[1:]
    for comb in itertools.combinations(rest, size - 1):
        s = (first,) + comb
        remaining = [x for x in rest if x not in comb]
        for p in partitions(remaining, size):
            yield [s] + p


def brute_best_score(devs, required, size):
    pad = (-len(devs)) % size
    items = list(devs) + [None] * pad
    best = None
    for p in partitions(items, size):
        ok = False
        for s in p:
            npad = sum(1 for x in s if x is None)
            if npad not in (0, pad):
                break
            if npad == 0 and all(r in s for r in required):
                ok = True
        else:
            if ok:
                sc = sum(set_score([x for x in s if x is not None]) for s in p)
                best = sc if best is None else max(best, sc)
    return best


def random_devices(rng, n):
    devs = [GpuDevice(index=i, uuid=f"GPU-{i:04x}", numa_node=rng.randint(0, 1)) for i in range(n)]
    for a in devs:
        for b in devs:
            if a.index < b.index:
                kind = rng.choice(["xgmi", "xgmi2", "pcie", "none"])
                lk = {"xgmi": [(IOLINK_XGMI, 15)], "xgmi2": [(IOLINK_XGMI, 15)] * 2,
                      "pcie": [(IOLINK_PCIE, 20)], "none": []}[kind]
                a.links[b.index] = list(lk)
                b.links[a.index] = list(lk)
    return devs


@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=1, max_value=7), st.integers(min_value=1, max_value=7), st.integers(0, 10**6),
       st.integers(0, 2))
def test_matches_exhaustive_objective(n, size, seed, nreq):
    rng = random.Random(seed)
    devs = random_devices(rng, n)
    size = min(size, n)
    required = rng.sample(devs, min(nreq, size))
    got = best_effort(devs, required, size)
    want = brute_best_score(devs, required, size)
    if want is None:
        assert got == []
        return
    assert len(got) == size and all(r in got for r in required) and None not in got
    rest = [d for d in devs if d not in got]
    rest_best = 0 if not rest else (brute_best_score(rest, [], size) if len(rest) >= size else 0)
    if len(rest) and len(rest) < size:
        rest_best = set_score(rest)
    assert set_score(got) + (rest_best or 0) == want


def test_mi355x_ubb_prefers_numa_locality():
    devs = FakeBackend(n=8, topology="xgmi", numa_split=4).devices()
    got = best_effort(devs, [], 4)
    assert {d.numa_node for d in got} == {0} or {d.numa_node for d in got} == {1}
    assert all(pair_score(a, b) == 101 for a, b in itertools.combinations(got, 2))


def test_required_device_is_honoured():
    devs = FakeBackend(n=8, topology="xgmi", numa_split=4).devices()
    got = best_effort(devs, [devs[5]], 2)
    assert devs[5] in got and len(got) == 2
    assert got[0].numa_node == got[1].numa_node == 1


def test_impossible_requests():
    devs = FakeBackend(n=2).devices()
    assert best_effort(devs, [], 3) == []
    assert best_effort(devs, devs, 1) == []
    assert best_effort(devs, [], 0) == []


def test_vgpu_preferred_allocation_maps_back():
    devs = FakeBackend(n=4, topology="pcie", numa_split=2).devices()
    vds = device_to_vdevices(devs, 2)
    avail = [v.id for v in vds]
    ids = allocate_vdevices(vds, avail, [], 2)
    assert len(ids) == 2
    phys = {i.rsplit("-", 1)[0] for i in ids}
    assert len(phys) == 2  # spread over two GPUs of one NUMA node
    nodes = {d.numa_node for d in devs if d.uuid in phys}
    assert len(nodes) == 1
    # must-include vGPU is kept (the reference would swap in the first vGPU of that GPU)
    must = vds[1].id
    ids = allocate_vdevices(vds, avail, [must], 2)
    assert must in ids


def test_vgpu_fallback_when_more_vgpus_than_gpus():
    vds = device_to_vdevices(FakeBackend(n=1).devices(), 4)
    ids = allocate_vdevices(vds, [v.id for v in vds], [], 3)
    assert ids == [v.id for v in vds[:3]]


def _sequential_pods(placement, pods, size=1, n=8, split=4):
    """The kubelet's view: each pod's GetPreferredAllocation sees the vGPUs still free."""
    vds = device_to_vdevices(FakeBackend(n=n, topology="xgmi").devices(), split)
    free = [v.id for v in vds]
    got = []
    for _ in range(pods):
        ids = allocate_vdevices(vds, free, [], size, placement=placement)
        assert len(ids) == size and all(i in free for i in ids)
        free = [i for i in free if i not in ids]
        got.append(ids)
    return got


def _gpu(vid):
    return vid.rsplit("-", 1)[0]


def test_spread_places_sequential_pods_on_distinct_gpus():
    pods = _sequential_pods("spread", 8)
    assert len({_gpu(p[0]) for p in pods}) == 8
    # a second round then fills every GPU's second slot before any third one
    more = _sequential_pods("spread", 16)
    per_gpu = {}
    for p in more:
        per_gpu[_gpu(p[0])] = per_gpu.get(_gpu(p[0]), 0) + 1
    assert sorted(per_gpu.values()) == [2] * 8


def test_binpack_fills_gpus_before_opening_new_ones():
    pods = _sequential_pods("binpack", 8)
    assert len({_gpu(p[0]) for p in pods}) == 2


def test_multi_vgpu_requests_keep_the_topology_score():
    """2-vGPU pods on a PCIe node (pairs score by NUMA node): every pod gets two distinct
    GPUs of one NUMA node, under both placements."""
    devs = FakeBackend(n=8, topology="pcie", numa_split=4).devices()
    by_uuid = {d.uuid: d for d in devs}
    for placement in ("spread", "binpack"):
        vds = device_to_vdevices(devs, 4)
        free = [v.id for v in vds]
        for _ in range(4):
            ids = allocate_vdevices(vds, free, [], 2, placement=placement)
            free = [i for i in free if i not in ids]
            g = [by_uuid[_gpu(i)] for i in ids]
            assert g[0] is not g[1] and g[0].numa_node == g[1].numa_node


def test_no_duplicate_gpu_while_another_gpu_is_free():
    """Two slots of one GPU are only preferred when fewer distinct GPUs are free."""
    vds = device_to_vdevices(FakeBackend(n=3, topology="xgmi").devices(), 4)
    # GPU 0 has all four slots free, GPUs 1 and 2 one slot each
    free = [v.id for v in vds if v.dev.index == 0] + [vds[4].id, vds[8].id]
    for placement in ("spread", "binpack"):
        ids = allocate_vdevices(vds, free, [], 3, placement=placement)
        assert len({_gpu(i) for i in ids}) == 3
    ids = allocate_vdevices(vds, free, [], 4)
    assert len(ids) == 4 and len({_gpu(i) for i in ids}) == 3  # one duplicate is unavoidable
    # two must-include vGPUs of one GPU are both kept
    ids = allocate_vdevices(vds, free, [vds[0].id, vds[1].id], 3)
    assert vds[0].id in ids and vds[1].id in ids and len(ids) == 3
