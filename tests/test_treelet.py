"""The treelet layout of the KD tree (csrc/host/treelet.cpp, the cooperative descent's records,
DESIGN.md §4) on the CPU: built from the host KD trees of the bench scenes (and of a one-leaf and
a depth-0 tree), every treelet position, exit and leaf slot is walked back into a tree, which must
equal the node tree branch for branch (split bits, axis, child order) and leaf for leaf (both
words), so a descent over treelets meets exactly the node descent's branches (kdtree.rs:66-104).
The checker is compiled from treelet.cpp with g++; no GPU."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_scene

CHECK = r"""
#include <cstdio>
#include <cstdint>
#include <vector>
#include "treelet.h"
using namespace rth;
static std::vector<uint32_t> N, T, L;
static long n_branch = 0, n_leaf = 0;
static int fail(const char* m, uint32_t a, uint32_t b) { std::printf("FAIL %s %u %u\n", m, a, b); return 1; }
// node i against treelet t, position p
static int cmp(uint32_t i, uint32_t t, uint32_t p) {
    const uint32_t* w = &T[16 * (size_t)t];
    const uint32_t tag = (w[7] >> (2 * p)) & 3u;
    const bool leaf = (N[2 * (size_t)i + 1] & 3u) == 3u;
    if (leaf) {
        if (tag != 3u || !((w[10] >> p) & 1u)) return fail("leaf tag", i, p);
        const uint32_t li = w[9] + __builtin_popcount(w[10] & ((1u << p) - 1u));
        if (L[2 * li] != N[2 * i] || L[2 * li + 1] != N[2 * i + 1]) return fail("leaf record", i, li);
        ++n_leaf;
        return 0;
    }
    if (tag != (N[2 * i + 1] & 3u) || w[p] != N[2 * i]) return fail("branch", i, p);
    ++n_branch;
    const uint32_t lo = N[2 * i + 1] >> 2;
    for (uint32_t c = 0; c < 2; ++c) {
        int r;
        if (p < 3) {
            r = cmp(lo + c, t, 2 * p + 1 + c);
        } else {
            const uint32_t k = 2 * (p - 3) + c, xb = (w[7] >> 14) & 0xffu;
            const bool cl = (N[2 * (size_t)(lo + c) + 1] & 3u) == 3u;
            if (((xb >> k) & 1u) == (cl ? 1u : 0u)) return fail("exit kind", i, k);
            if (!cl) {
                const uint32_t tc = w[8] + __builtin_popcount(xb & ((1u << k) - 1u));
                if (16 * (size_t)tc >= T.size()) return fail("child treelet", i, tc);
                r = cmp(lo + c, tc, 0);
            } else {
                if (!((w[10] >> (7 + k)) & 1u)) return fail("exit leaf bit", i, k);
                const uint32_t li = w[9] + __builtin_popcount(w[10] & ((1u << (7 + k)) - 1u));
                if (L[2 * li] != N[2 * (lo + c)] || L[2 * li + 1] != N[2 * (lo + c) + 1]) return fail("exit leaf", i, li);
                ++n_leaf;
                r = 0;
            }
        }
        if (r) return r;
    }
    return 0;
}
int main(int argc, char** argv) {
    FILE* f = std::fopen(argv[1], "rb");
    uint32_t v;
    while (std::fread(&v, 4, 1, f) == 1) N.push_back(v);
    std::fclose(f);
    if (!build_treelets(N, &T, &L)) return fail("build", 0, 0);
    if (T.size() % 16) return fail("record size", (uint32_t)T.size(), 0);
    for (size_t t = 0; t < T.size() / 16; ++t)
        for (int k = 11; k < 16; ++k) if (T[16 * t + k]) return fail("padding", (uint32_t)t, k);
    if (cmp(0, 0, 0)) return 1;
    // every leaf record and every treelet is reached exactly once
    long reached_leaves = (long)L.size() / 2;
    std::printf("OK treelets=%zu leaves=%zu branches=%ld visited_leaves=%ld\n", T.size() / 16, L.size() / 2, n_branch, n_leaf);
    return n_leaf == reached_leaves ? 0 : fail("leaf count", (uint32_t)n_leaf, (uint32_t)reached_leaves);
}
"""


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    d = tmp_path_factory.mktemp("treelet")
    src = d / "check.cpp"
    src.write_text(CHECK)
    host = os.path.join(ROOT, "gpu-ray_trace-rust_amd", "csrc", "host")
    exe = str(d / "check")
    r = subprocess.run(["g++", "-O2", "-std=c++17", f"-I{host}", "-o", exe, str(src), os.path.join(host, "treelet.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe, d


def run_check(checker, nodes):
    exe, d = checker
    path = d / "nodes.bin"
    np.ascontiguousarray(nodes, dtype=np.uint32).tofile(path)
    r = subprocess.run([exe, str(path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("name,depth", [("walled", 17), ("biplane", None), ("spaceship_r1", None), ("a380", None),
                                        ("triangles", None), ("walled", 0), ("walled", 1), ("walled", 4)])
def test_treelets_equal_node_tree(checker, name, depth):
    from rt_amd import render

    sc = load_scene(name)
    kd = render.KdTree(sc.desc, int(sc.info.kd_tree_depth) if depth is None else depth)
    out = run_check(checker, np.asarray(kd.nodes, dtype=np.uint32).reshape(-1))
    print(name, out)


def test_single_leaf_tree(checker):
    """A tree of one leaf (triangles.yml at depth 0): one treelet whose position 0 is the leaf."""
    nodes = np.array([[5, (7 << 2) | 3]], dtype=np.uint32)
    out = run_check(checker, nodes.reshape(-1))
    assert "treelets=1 leaves=1" in out
