"""The multi-device host plan on CPU (no GPU call): the LZF_GPU_DEVICES
grammar and the partition rule the host-memory calls use -- value i goes to
plan entry i mod G, entry g's values in increasing order,
so the results it writes back land at the caller's indices."""
import pytest

import gibson_amd


@pytest.mark.parametrize("count", [0, 1, 2, 3, 7, 8, 9, 1000, 262144, 262147])
@pytest.mark.parametrize("groups", [1, 2, 3, 8])
def test_split_is_round_robin(count, groups):
    seen = []
    for g in range(groups):
        first, stride, n = gibson_amd.host_split(count, groups, g)
        assert (first, stride) == (g, groups)
        vals = [first + k * stride for k in range(n)]
        assert vals == [i for i in range(count) if i % groups == g]
        seen += vals
    assert sorted(seen) == list(range(count))


def test_split_outside_the_plan_is_empty():
    assert gibson_amd.host_split(10, 4, 4)[2] == 0
    assert gibson_amd.host_split(10, 0, 0)[2] == 0
    assert gibson_amd.host_split(3, 8, 5)[2] == 0


@pytest.mark.parametrize("count", [0, 1, 2, 3, 7, 8, 9, 1000, 262144, 262147, 4194304])
@pytest.mark.parametrize("groups", [1, 2, 3, 8])
def test_split_block_is_contiguous(count, groups):
    # LZF_GPU_SPLIT=block: entry g takes [floor(count g / G), floor(count (g+1) / G)),
    # the spans abut in entry order and cover the batch once; sizes differ by
    # at most one value
    end, sizes = 0, []
    for g in range(groups):
        first, n = gibson_amd.host_split_block(count, groups, g)
        assert first == count * g // groups == end
        assert n == count * (g + 1) // groups - first
        end = first + n
        sizes.append(n)
    assert end == count
    assert max(sizes) - min(sizes) <= 1


def test_split_block_outside_the_plan_is_empty():
    assert gibson_amd.host_split_block(10, 4, 4)[1] == 0
    assert gibson_amd.host_split_block(10, 0, 0)[1] == 0


@pytest.mark.parametrize("env,want", [(None, "round-robin"), ("rr", "round-robin"), ("block", "block")])
def test_split_policy_from_env(env, want, monkeypatch):
    if env is None:
        monkeypatch.delenv("LZF_GPU_SPLIT", raising=False)
    else:
        monkeypatch.setenv("LZF_GPU_SPLIT", env)
    assert gibson_amd.host_split_policy() == want


def test_gather_order_restores_the_batch():
    # a stand-in for the workers: each entry "processes" its share in its own
    # order and writes result i at index i -- the caller's array comes back whole
    count, groups = 1003, 3
    res = [None] * count
    for g in reversed(range(groups)):
        first, stride, n = gibson_amd.host_split(count, groups, g)
        for k in reversed(range(n)):
            i = first + k * stride
            res[i] = (g, i)
    assert all(r is not None and r[1] == i and r[0] == i % groups for i, r in enumerate(res))


@pytest.mark.parametrize("spec,visible,want", [
    ("0", 1, [0]),
    ("0,0", 1, [0, 0]),
    ("0, 1,3", 4, [0, 1, 3]),
    ("all", 8, list(range(8))),
    ("all", 1, [0]),
])
def test_device_list_grammar(spec, visible, want):
    assert gibson_amd.parse_device_list(spec, visible) == want


@pytest.mark.parametrize("spec,visible,code", [
    ("1", 1, -3),          # past the visible devices: ENODEV
    ("all", 0, -3),
    ("", 4, -1),           # empty: EARG
    ("0;1", 4, -1),
    ("x", 4, -1),
    ("-1", 4, -3),
])
def test_device_list_rejects(spec, visible, code):
    assert gibson_amd.parse_device_list(spec, visible) == code
