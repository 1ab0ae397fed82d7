"""bench.py's warm-up through the timed graph's own executable
(bench.warm_passes): the positions chosen run exactly W steps, on the inputs
``step(0 .. W-1)`` would use, one use per position per replay."""
import bench


def _check(w, n, i0, rot):
    passes = bench.warm_passes(w, n, i0, rot)
    assert sum(map(len, passes)) == w
    for p in passes:
        assert len(set(p)) == len(p) and all(0 <= j < n for j in p)
    return passes


def test_same_inputs_as_warmup_steps():
    # eth_hotel_synth at the driver's invocation: 16 rotated batches, W 5, K 20
    (p,) = _check(5, 20, 5, 16)
    assert sorted((5 + j) % 16 for j in p) == [0, 1, 2, 3, 4]


def test_more_warmup_than_steps():
    passes = _check(50, 20, 50, 16)
    assert len(passes) == 4          # batch 0: four uses, one timed position
    got = sorted((50 + j) % 16 for p in passes for j in p)
    assert got == sorted(i % 16 for i in range(50))


def test_inputs_not_in_timed_steps():
    # 64 batches, 4 timed steps: the warm-up's inputs never occur; any W positions
    passes = _check(3, 4, 3, 64)
    assert passes == [[0, 1, 2]]


def test_no_warmup():
    assert bench.warm_passes(0, 20, 1, 16) == []
