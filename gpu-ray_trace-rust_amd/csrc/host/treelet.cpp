// treelet.cpp — 3-level treelets of the KD tree (treelet.h).  The tree is the one rt_kd_build
// makes (KdTree::build, kdtree.rs:26-56 / 107-137); only its layout changes.
#include "treelet.h"

#include <cstddef>

namespace rth {

namespace {
constexpr uint32_t LEAF = 3u;
inline bool is_leaf(const std::vector<uint32_t>& n, uint32_t i) { return (n[2 * (size_t)i + 1] & 3u) == LEAF; }
inline uint32_t low_child(const std::vector<uint32_t>& n, uint32_t i) { return n[2 * (size_t)i + 1] >> 2; }
}  // namespace

bool build_treelets(const std::vector<uint32_t>& nodes, std::vector<uint32_t>* treelets,
                    std::vector<uint32_t>* leaves) {
    if (nodes.size() < 2) return true;
    // breadth first over treelet roots; a root's index is its position in this list
    std::vector<uint32_t> roots{0u};
    for (size_t t = 0; t < roots.size(); ++t) {
        if (roots.size() >= (1u << 29)) return false;
        uint32_t pos[7], w[TREELET_WORDS] = {};
        bool present[7] = {};
        pos[0] = roots[t];
        present[0] = true;
        uint32_t tags = 0, xb = 0, leafmask = 0;
        uint32_t exit_node[8] = {};
        for (uint32_t p = 0; p < 7; ++p) {
            if (!present[p]) {
                tags |= LEAF << (2 * p);  // never visited
                continue;
            }
            const uint32_t i = pos[p];
            if (is_leaf(nodes, i)) {
                tags |= LEAF << (2 * p);
                leafmask |= 1u << p;
                continue;
            }
            w[p] = nodes[2 * (size_t)i];
            tags |= (nodes[2 * (size_t)i + 1] & 3u) << (2 * p);
            const uint32_t lo = low_child(nodes, i);
            for (uint32_t c = 0; c < 2; ++c) {
                if (p < 3) {
                    pos[2 * p + 1 + c] = lo + c;
                    present[2 * p + 1 + c] = true;
                } else {
                    const uint32_t k = 2 * (p - 3) + c;
                    exit_node[k] = lo + c;
                    if (is_leaf(nodes, lo + c)) leafmask |= 1u << (7 + k);
                    else xb |= 1u << k;
                }
            }
        }
        w[7] = tags | (xb << 14);
        w[8] = (uint32_t)roots.size();  // the children are appended next, in exit order
        w[9] = (uint32_t)(leaves->size() / 2);
        w[10] = leafmask;
        for (uint32_t s = 0; s < 15; ++s) {
            if (!((leafmask >> s) & 1u)) continue;
            const uint32_t i = s < 7 ? pos[s] : exit_node[s - 7];
            leaves->push_back(nodes[2 * (size_t)i]);
            leaves->push_back(nodes[2 * (size_t)i + 1]);
        }
        for (uint32_t k = 0; k < 8; ++k)
            if ((xb >> k) & 1u) roots.push_back(exit_node[k]);
        treelets->insert(treelets->end(), w, w + TREELET_WORDS);
    }
    return true;
}

}  // namespace rth
