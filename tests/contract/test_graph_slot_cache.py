"""Decoder-step graph cache bookkeeping (runtime/summarize._SlotCache), CPU only.

The GPU tests (tests/kernels/test_decode_gpu.py -k graph_cache) check that replayed steps
are bit-identical; here: admission, LRU eviction by count and by bytes, busy slots kept,
per-model caches."""
import torch

from agent_tpu_amd.runtime.summarize import _Slot, _SlotCache, slot_cache


def _slot(key, nbytes, graph=True):
    sl = _Slot(key)
    sl.bufs["x"] = torch.empty(nbytes, dtype=torch.uint8)
    sl.graph = object() if graph else None
    return sl


def _release(sc, sl):  # _SlotCache.release records a HIP event; the CPU test only frees the slot
    sl.busy = False


def test_admit_evicts_idle_lru_by_count():
    sc = _SlotCache()
    sc.max_slots, sc.max_bytes = 2, 1 << 20
    a, b, c = _slot("a", 10), _slot("b", 10), _slot("c", 10)
    assert sc.admit(a) and sc.admit(b)
    _release(sc, a)
    _release(sc, b)
    a.last, b.last = 1.0, 2.0  # a is the least recently used
    assert sc.admit(c)
    assert [s.key for s in sc.slots] == ["b", "c"]


def test_busy_slots_are_never_evicted():
    sc = _SlotCache()
    sc.max_slots, sc.max_bytes = 1, 1 << 20
    a = _slot("a", 10)
    assert sc.admit(a)  # admitted slots start busy (their search holds them)
    assert not sc.admit(_slot("b", 10))  # full of busy slots: runs uncached
    assert [s.key for s in sc.slots] == ["a"]


def test_byte_budget():
    sc = _SlotCache()
    sc.max_slots, sc.max_bytes = 8, 100
    assert not sc.admit(_slot("huge", 101))  # larger than the whole budget
    a = _slot("a", 60)
    assert sc.admit(a)
    _release(sc, a)
    assert sc.admit(_slot("b", 60))  # evicts a to fit
    assert [s.key for s in sc.slots] == ["b"] and sc.nbytes() == 60


def test_acquire_matches_key_and_idle_captured_slots():
    sc = _SlotCache()
    a = _slot("k", 10)
    assert sc.admit(a)
    assert sc.acquire("k") is None  # busy
    _release(sc, a)
    assert sc.acquire("other") is None
    got = sc.acquire("k")
    assert got is a and a.busy and sc.hits == 1 and sc.misses == 2
    a.busy = False
    a.graph = None  # never captured: not reusable
    assert sc.acquire("k") is None


def test_cache_lives_on_the_model():
    class M:
        pass

    m1, m2 = M(), M()
    assert slot_cache(m1) is slot_cache(m1) and slot_cache(m1) is not slot_cache(m2)
