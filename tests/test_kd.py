"""The host KD build (rt_kd_build, breadth-first 8-byte nodes) equals the oracle's recursive
restatement of KdTree::build (kdtree.rs:26-56,107-137) node for node and ref for ref."""
import numpy as np
import pytest

from conftest import load_scene


def compare(scene, depth, oracle):
    from rt_amd import render

    kd = render.KdTree(scene.desc, depth)
    rows, refs = kd.canonical_dfs()
    orows, orefs, obounds = oracle.kd_dump(scene.desc, depth)
    assert np.array_equal(rows, orows)
    assert np.array_equal(refs, orefs)
    assert np.array_equal(obounds, kd.bounds)
    return kd


def test_walled_full_tree(oracle, walled):
    kd = compare(walled, 17, oracle)
    rows, _ = kd.canonical_dfs()
    # full depth-17 tree (rows = reachable nodes; the array adds padding)
    assert (len(rows), kd.n_refs, kd.max_leaf_depth) == (524287, 786443, 18)
    leaves = rows[:, 0] == 1
    assert leaves.sum() == 262144
    assert rows[leaves, 2].max() == 9


@pytest.mark.parametrize("depth", [0, 1, 2, 5, 9])
def test_walled_depths(oracle, walled, depth):
    compare(walled, depth, oracle)


def test_blocked_layout(walled):
    """128-byte blocks (16 nodes): a child pair lies in its parent's block or starts a block,
    so a root-to-leaf descent of the depth-18 tree touches at most 1 + ceil(15 / 3) = 6 lines."""
    from rt_amd import render

    kd = render.KdTree(walled.desc, 17)
    assert kd.n_nodes % 16 == 0
    lines_on_path = {0: 1}
    stack = [0]
    worst = 0
    while stack:
        i = stack.pop()
        a, b = kd.nodes[i]
        if (b & 3) == 3:
            worst = max(worst, lines_on_path[i])
            continue
        low = int(b >> 2)
        assert low % 2 == 0 or low // 16 == i // 16
        same = low // 16 == i // 16
        assert same or low % 16 == 0, "a child pair outside the parent's block must start a block"
        for c in (low, low + 1):
            lines_on_path[c] = lines_on_path[i] + (0 if same else 1)
            stack.append(c)
    assert worst <= 6, worst


def test_single_and_empty_scenes(oracle):
    """len <= 1 makes a leaf immediately (kdtree.rs:109)."""
    import copy
    from rt_amd import scheme

    base = scheme.load_json(__import__("conftest").SCENES + "/walled.json")
    one = copy.deepcopy(base)
    one["scene_members"] = one["scene_members"][:1]
    sc = scheme.load(one)
    kd = compare(sc, 17, oracle)
    assert len(kd.canonical_dfs()[0]) == 1 and kd.n_refs == 1


@pytest.mark.parametrize("name", ["walled", "biplane", "spaceship_r1", "a380", "triangles"])
def test_parallel_build_is_byte_identical(monkeypatch, name):
    """rt_kd_build builds the subtrees below its top levels on several threads and renumbers the
    whole tree breadth first: the node and ref arrays equal the single-threaded build's (the
    sequential breadth-first numbering) byte for byte."""
    from rt_amd import render

    sc = load_scene(name)
    depth = int(sc.info.kd_tree_depth)
    monkeypatch.setenv("RT_DEBUG_KD_THREADS", "1")
    one = render.KdTree(sc.desc, depth)
    monkeypatch.setenv("RT_DEBUG_KD_THREADS", "8")
    par = render.KdTree(sc.desc, depth)
    assert np.array_equal(one.nodes, par.nodes)
    assert np.array_equal(one.refs, par.refs)
    assert one.max_leaf_depth == par.max_leaf_depth and np.array_equal(one.bounds, par.bounds)


@pytest.mark.parametrize("name,threads", [("walled", "1"), ("biplane", "8")])
def test_build_budget_returns_oom(monkeypatch, name, threads):
    """The build stops with RT_ERR_OOM once its nodes or refs reach the budget (2^30 in the
    product, RT_DEBUG_KD_BUDGET lowers it), on one thread (walled) and in the threaded subtree
    builds (biplane: 7,316 triangles), instead of growing to the end; a later build with the
    default budget is unaffected."""
    from rt_amd import abi, render

    sc = load_scene(name)
    depth = int(sc.info.kd_tree_depth)
    full = render.KdTree(sc.desc, depth)
    monkeypatch.setenv("RT_DEBUG_KD_THREADS", threads)
    monkeypatch.setenv("RT_DEBUG_KD_BUDGET", str(min(full.n_nodes, full.n_refs) // 2))
    with pytest.raises(abi.RtError) as e:
        render.KdTree(sc.desc, depth)
    assert e.value.status == abi.RT_ERR_OOM
    monkeypatch.delenv("RT_DEBUG_KD_BUDGET")
    again = render.KdTree(sc.desc, depth)
    assert np.array_equal(again.refs, full.refs) and np.array_equal(again.nodes, full.nodes)
