"""The oracle's two accumulation orders agree under direct-light sampling (radiance.rs:46-56,
89-120), including towards a DiffSpec emitter, whose hit_info draws one uniform
(sphere.rs:76, uniform_diff_spec.rs:33-36).  The reference draws it only after the recursive
subtree below the vertex, so it shifts no path draw; the forward order must keep it so."""
import json
import os

import numpy as np

import parity
from conftest import SCENES


def _walled_dls(emitter_divert=None):
    from rt_amd import scheme

    d = json.load(open(os.path.join(SCENES, "walled.json")))
    for m in d["scene_members"]:
        mat = m.get("!Sphere", {}).get("mat", {})
        if "emissive" in mat and emitter_divert is not None:
            mat["divert_ray"] = emitter_divert
    d["render_info"]["rad_info"]["dir_light_samp"] = True
    d["render_info"]["width"], d["render_info"]["height"] = 120, 60
    return scheme.load(d)


def _check(oracle, sc):
    tiles = [(40, 20, 40, 20)]
    f = oracle.render(sc, tiles, 0, 6, accum=oracle.ACCUM_FORWARD, threads=4)
    r = oracle.render(sc, tiles, 0, 6, accum=oracle.ACCUM_RECURSIVE, threads=4)
    s = parity.stats(f, r)
    assert s["frac_ok"] >= parity.MIN_FRAC, s
    assert s["mean_rel_err"] < 1e-4, s
    return f


def test_forward_equals_recursive_with_dls(oracle):
    _check(oracle, _walled_dls())


def test_forward_equals_recursive_with_diffspec_emitter(oracle):
    f = _check(oracle, _walled_dls({"!DiffSpec": {"diffp": 0.6}}))
    plain = _check(oracle, _walled_dls())
    assert not np.array_equal(f, plain)  # the emitters' material does change the image
