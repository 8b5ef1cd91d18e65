"""Where the reference traversal's descent steps fall in the KD tree: branch-node visits of
KdTree::stack_search (kdtree.rs:73-89) by depth, from the oracle's counted render (forward
radiance, the device's path order) on a grid of pixels.  The share of visits in the top L levels
bounds what a top-of-tree node cache of L levels (2^L - 1 nodes, LDS or SGPRs) could take off
the vector-memory pipeline: the device makes one node-pair load per branch step of its
cooperative descent (RT_PAIR_FETCH).
Usage: python tools/descent_depths.py [scene[:spp] ...] > profiles/r4_descent_depths.jsonl"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main(specs):
    import oracle_py
    from rt_amd import scheme

    for spec in specs:
        name, _, spp = spec.partition(":")
        spp = int(spp or 2)
        sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", name + ".json"))
        loaded = scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"))
        w, h = int(loaded.info.width), int(loaded.info.height)
        tiles = [(x, y, 1, 1) for y in range(0, h, 8) for x in range(0, w, 8)]
        oracle_py.mix_counts(reset=True)
        _, cnt = oracle_py.render(loaded, tiles, 0, spp, accum=oracle_py.ACCUM_FORWARD, counts=True)
        mix = oracle_py.mix_counts(reset=True)
        by_depth = [mix[f"node_d{d}"] for d in range(40)]
        total = sum(by_depth)
        samples = len(tiles) * spp
        cum, top = 0, {}
        for d, v in enumerate(by_depth):
            cum += v
            top[d + 1] = round(cum / total, 4) if total else None
        print(json.dumps({"scene": name, "spp": spp, "pixels": len(tiles), "kd_depth": int(loaded.info.kd_tree_depth),
                          "branch_visits_per_sample": round(total / samples, 2),
                          "leaf_visits_per_sample": round((cnt["nodes"] - total) / samples, 2),
                          "share_in_top_levels": {k: v for k, v in top.items() if k in (4, 6, 8, 10, 12, 14)},
                          "by_depth_per_sample": [round(v / samples, 3) for v in by_depth[:24]]}), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["a380:1", "biplane:1", "spaceship_r1:1"])
