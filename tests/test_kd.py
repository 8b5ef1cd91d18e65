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
    # full depth-17 tree
    assert (kd.n_nodes, kd.n_refs, kd.max_leaf_depth) == (524287, 786443, 18)
    leaves = (kd.nodes[:, 1] & 3) == 3
    assert leaves.sum() == 262144
    assert kd.nodes[leaves, 0].max() == 9


@pytest.mark.parametrize("depth", [0, 1, 2, 5, 9])
def test_walled_depths(oracle, walled, depth):
    compare(walled, depth, oracle)


def test_bfs_layout_levels_are_prefix(walled):
    """Children are allocated in pairs in breadth-first order: the top levels form a prefix
    of the node array (the device stages that prefix in LDS)."""
    from rt_amd import render

    kd = render.KdTree(walled.desc, 17)
    depth = np.zeros(kd.n_nodes, np.int64)
    for i in range(kd.n_nodes):
        a, b = kd.nodes[i]
        if (b & 3) != 3:
            depth[(b >> 2)] = depth[i] + 1
            depth[(b >> 2) + 1] = depth[i] + 1
    assert np.all(np.diff(depth) >= 0)


def test_single_and_empty_scenes(oracle):
    """len <= 1 makes a leaf immediately (kdtree.rs:109)."""
    import copy
    from rt_amd import scheme

    base = scheme.load_json(__import__("conftest").SCENES + "/walled.json")
    one = copy.deepcopy(base)
    one["scene_members"] = one["scene_members"][:1]
    sc = scheme.load(one)
    kd = compare(sc, 17, oracle)
    assert kd.n_nodes == 1 and kd.n_refs == 1
