// treelet.h — the KD tree re-laid as 3-level treelets for the cooperative descent of the general
// queue kernel (trace.hip stack_search_coop).  Host only; no HIP types, so the CPU
// tests compile it on its own (tests/test_treelet.py).
//
// A treelet is a node and the two levels below it: 7 positions in heap order (0 the root, 1 / 2 its
// low / high child, 3..6 the grandchildren) and 8 exits, the children of positions 3..6 (exit
// 2 (p - 3) + c, c = 0 low / 1 high).  Its record is 64 B (one half of a 128-B line), of which the
// device loads the first 48 B in three 16-B loads:
//   w[0..6]  split bits of the branches at positions 0..6 (0 where the position is a leaf or absent)
//   w[7]     bits 2p..2p+1: axis of the branch at position p, 3 for a leaf (or absent);
//            bits 14..21: exit k is a branch (the root of another treelet)
//   w[8]     index of the first child treelet: exit k's treelet is w[8] + popcount(branch exits < k)
//   w[9]     index of the treelet's first leaf in the leaf array
//   w[10]    bit s set when slot s is a leaf (slots 0..6 positions, 7..14 exits); slot s's leaf is
//            w[9] + popcount(leaf slots < s)
//   w[11..15] zero
// Leaves keep the node layout {count | leading spheres << 24, (ref offset << 2) | 3}.  Treelets are
// numbered breadth first, so the child treelets of one treelet are consecutive.  The splits, axes
// and child order are the tree's own: a descent over treelets meets the same branches, in the same
// order, with the same split values as one over the nodes (kdtree.rs:66-104).
#pragma once

#include <cstdint>
#include <vector>

namespace rth {

constexpr uint32_t TREELET_WORDS = 16;

// nodes: 2 words per node {a, b}; a branch is {split bits, (low child << 2) | axis} with its
// children at low and low + 1, a leaf {count word, (offset << 2) | 3}; node 0 is the root.
// Appends the treelet records (TREELET_WORDS words each) and the leaf records (2 words each).
// Returns false when the tree has more treelets than 2^29 (a treelet index and a position share a
// 32-bit stack entry on the device).
bool build_treelets(const std::vector<uint32_t>& nodes, std::vector<uint32_t>* treelets,
                    std::vector<uint32_t>* leaves);

}  // namespace rth
