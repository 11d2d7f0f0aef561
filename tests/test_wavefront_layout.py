"""CPU: the wavefront schedule's queue layout (csrc/rt_wavefront.hpp, wf_pos) -- streams of 64-entry
blocks, entry k of stream v at (v + (k // 64) * G) * 64 + k % 64 -- keeps every stream's entries
inside the queue and disjoint from every other stream's, for any stream count G and any counts a
shade launch can produce (never more than the stream held at bounce 0).  A Python restatement of
the index arithmetic; the GPU tests (test_wavefront.py) check the rendered bits."""
import numpy as np
import pytest


def wf_pos(v, k, G):
    return (v + (k >> 6) * G) * 64 + (k & 63)


def stream_capacity(v, n_blocks, G):
    """entries of stream v at bounce 0: its blocks v, v + G, ... below n_blocks, 64 each"""
    return ((n_blocks - v + G - 1) // G if n_blocks > v else 0) * 64


@pytest.mark.parametrize("n_blocks,G", [(1, 1), (7, 3), (129600, 1536), (1036800, 1536), (5000, 2048),
                                        (64, 64), (65, 64), (100, 1)])
def test_streams_fill_the_queue_exactly(n_blocks, G):
    cap = n_blocks * 64
    seen = np.zeros(cap, np.uint8)
    for v in range(min(G, n_blocks)):
        n = stream_capacity(v, n_blocks, G)
        k = np.arange(n, dtype=np.int64)
        p = wf_pos(v, k, G)
        assert p.max() < cap
        seen[p] += 1
    assert (seen == 1).all(), "every queue position belongs to exactly one stream entry"


@pytest.mark.parametrize("seed", range(5))
def test_compacted_counts_stay_inside_the_stream(seed):
    rng = np.random.default_rng(seed)
    n_blocks, G = int(rng.integers(1, 5000)), int(rng.integers(1, 700))
    cap = n_blocks * 64
    owner = np.full(cap, -1, np.int64)
    for v in range(min(G, n_blocks)):
        full = stream_capacity(v, n_blocks, G)
        c = int(rng.integers(0, full + 1))  # a later bounce: any count up to the bounce-0 count
        p = wf_pos(v, np.arange(c, dtype=np.int64), G)
        assert (p < cap).all()
        assert (owner[p] == -1).all()
        owner[p] = v
        # a stream's entries sit in its own blocks
        assert ((p // 64) % G == v).all()


def test_units_cover_every_entry_once():
    """extend walks units u = j * G + v (block j of stream v) for u < G * ceil(max_count / 64):
    the units with j * 64 < count_v hold exactly the stream's entries"""
    rng = np.random.default_rng(7)
    n_blocks, G = 3000, 256
    counts = [int(rng.integers(0, stream_capacity(v, n_blocks, G) + 1)) for v in range(G)]
    n_units = G * ((max(counts) + 63) // 64)
    got = []
    for u in range(n_units):
        j, v = divmod(u, G)
        c = counts[v]
        n = min(64, c - j * 64) if c > j * 64 else 0
        got.extend(wf_pos(v, j * 64 + np.arange(n), G).tolist())
    want = [p for v in range(G) for p in wf_pos(v, np.arange(counts[v]), G).tolist()]
    assert sorted(got) == sorted(want) and len(got) == len(set(got))
