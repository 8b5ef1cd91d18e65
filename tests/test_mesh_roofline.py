"""The mesh configs' roofline (tools/mesh_roofline.py, bench.py roofline(model_config=...)) is
recomputable from committed profiles alone: the vector-memory issue ceiling is
the sum over load classes of wave-loads x the measured gather cost of their shape (the committed
gather sweep), the latency ceiling is resident waves over dependent load steps x unloaded latency,
and bench.py's fractions are achieved / ceiling with the larger fraction named as the bound.
CPU only: every input is a committed file."""
import json
import math
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)


def _entries():
    import glob

    out = []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_vmem_lines.jsonl"))):
        for line in open(p):
            if line.strip():
                d = json.loads(line)
                if "lines_by_class" in d:
                    out.append((d, os.path.relpath(p, ROOT)))
    return out


def test_gather_sweep_is_committed_and_monotone():
    """The sweep covers every record kind the model prices, at 16 / 32 / 64 active lanes, from an
    L1- and an L2-resident table; a wave-load touching more lines never costs less at 64 lanes
    from L2 (the fill path)."""
    import mesh_roofline

    sw, src = mesh_roofline.sweep_table()
    assert sw and src.startswith("profiles/")
    for kind in ("dword", "dwordx2", "dwordx4", "tri48"):
        for level in ("L1", "L2"):
            for lanes in (16, 32, 64):
                assert (kind, level, lanes) in sw, (kind, level, lanes)
        pts = sw[(kind, "L2", 64)]
        costs = [t for _, t in pts]
        assert costs[-1] > 2.5 * costs[0], pts  # 64 random lines from L2 cost far more than one line


@pytest.mark.parametrize("idx", range(3))
def test_model_recomputes_from_its_inputs(idx):
    import mesh_roofline

    ents = _entries()
    if idx >= len(ents):
        pytest.skip("fewer committed load-class measurements")
    vl, vsrc = ents[idx]
    scene = vl["scene"]
    c = mesh_roofline.counters_for(scene)
    assert c, scene
    m = mesh_roofline.model_from(vl, vsrc, c[0], c[1])
    vi, la = m["vmem_issue"], m["latency"]
    # ceiling_v = 1 / sum_c wl_c (h1 / R_L1 + (1 - h1) / R_L2)
    t = sum(x["ns_per_sample"] for x in vi["classes"].values())
    assert math.isclose(t, vi["ns_per_sample"], rel_tol=2e-3)
    assert math.isclose(vi["ceiling_Msamples_s"], 1e3 / vi["ns_per_sample"], rel_tol=2e-3)
    h1 = vi["l1_line_hit_frac"]
    for x in vi["classes"].values():
        assert math.isclose(x["ns_per_sample"], x["wave_loads"] * (h1 * x["ns_L1"] + (1 - h1) * x["ns_L2"]),
                            rel_tol=2e-3, abs_tol=1e-4)
    # ceiling_l = W / (S x L)
    assert math.isclose(la["ceiling_Msamples_s"], la["resident_waves"] / (la["steps_per_sample"] * la["ns_per_step"]) * 1e3,
                        rel_tol=2e-3)
    assert 0.0 <= h1 <= 1.0 and vi["ceiling_Msamples_s"] > 0 and la["ceiling_Msamples_s"] > 0


def test_bench_roofline_uses_the_model(monkeypatch):
    """bench.roofline with a model config: achieved = samples per launch / kernel time, the two
    ceilings as candidates in Msamples/s, TD / TA busy only as secondary fields, and the bound the
    larger fraction (here forced: counters and load classes of one committed pair)."""
    import bench
    import mesh_roofline

    ents = [e for e in _entries() if mesh_roofline.counters_for(e[0]["scene"])]
    if not ents:
        pytest.skip("no committed load classes with counters")
    vl, vsrc = ents[0]
    cnt, csrc = mesh_roofline.counters_for(vl["scene"])
    bid = cnt["build_id"]
    monkeypatch.setattr(bench, "committed_counters", lambda b, s, n: (cnt, csrc))
    monkeypatch.setattr(mesh_roofline, "vmem_entry", lambda config, build_id=None: (vl, vsrc))
    per_launch = cnt["samples_per_launch"]
    kms = 25.0
    r = bench.roofline(vl["scene"], per_launch, kms, bid, "k", "test", model_config=vl.get("config", vl["scene"]))
    ach = per_launch / (kms * 1e-3) / 1e6
    m = mesh_roofline.model_from(vl, vsrc, cnt, csrc)
    for key in ("vmem_issue", "latency"):
        assert r[key]["unit"] == "Msamples/s"
        assert math.isclose(r[key]["achieved"], ach, rel_tol=1e-3)
        assert r[key]["peak"] == m[key]["ceiling_Msamples_s"]
        assert math.isclose(r[key]["frac"], ach / m[key]["ceiling_Msamples_s"], rel_tol=1e-3)
    assert "vmem" not in r and r["vmem_units"]["td_busy_frac"] == cnt["td_busy_frac"]
    cands = {k: r[k]["frac"] for k in ("valu", "hbm", "vmem_issue", "latency") if k in r}
    if r["bound"] is not None:
        assert r["bound"] == max(cands, key=cands.get)
