"""Per-pixel comparison used by the -m gpu parity tests (tolerances stated in DESIGN.md §Parity).

Gate: per-pixel L-inf over RGB <= REL_TOL * max(1, |ref|) on at least
MIN_FRAC of the pixels.  Against the forward oracle the device is bit-identical (glibc's
transcendentals restated in include/rt_libm.h); against the recursive oracle only the
accumulation order differs.  Any pixel outside the gate would be a path-divergent branch flip:
they are counted, not hidden.
"""
import numpy as np

REL_TOL = 1e-4
MIN_FRAC = 0.999


def stats(gpu: np.ndarray, ref: np.ndarray) -> dict:
    g, r = gpu[:, :3].astype(np.float64), ref[:, :3].astype(np.float64)
    d = np.abs(g - r).max(axis=1)
    scale = np.maximum(1.0, np.abs(r).max(axis=1))
    ok = d <= REL_TOL * scale
    exact = np.all(gpu[:, :3] == ref[:, :3], axis=1)
    return {"n": int(len(d)), "frac_ok": float(ok.mean()), "frac_exact": float(exact.mean()),
            "max_abs": float(d.max()) if len(d) else 0.0, "n_out": int((~ok).sum()),
            "mean_rel_err": float(np.abs(g.mean(0) - r.mean(0)).max() / max(1e-12, np.abs(r.mean(0)).max()))}


def u8(img: np.ndarray) -> np.ndarray:
    f = np.clip(img[:, :3], 0, 1) * np.float32(255) + np.float32(0.5)
    return np.nan_to_num(np.trunc(f), nan=0).astype(np.int32)


def frac_u8_within(gpu, ref, lsb=1):
    return float((np.abs(u8(gpu) - u8(ref)).max(axis=1) <= lsb).mean())


def worst_pixel(gpu: np.ndarray, ref: np.ndarray) -> dict:
    """The pixel farthest outside (or nearest the edge of) the gate, for the test log."""
    g, r = gpu[:, :3].astype(np.float64), ref[:, :3].astype(np.float64)
    d = np.abs(g - r).max(axis=1) / np.maximum(1.0, np.abs(r).max(axis=1))
    i = int(np.argmax(d)) if len(d) else 0
    return {"index": i, "rel_err": float(d[i]) if len(d) else 0.0,
            "gpu": gpu[i, :3].tolist() if len(d) else None, "ref": ref[i, :3].tolist() if len(d) else None}


def assert_reference_order(gpu: np.ndarray, ref_recursive: np.ndarray, label: str = "") -> dict:
    """The stated gate against the reference's own recursive accumulation order (radiance.rs:44,59;
    SURVEY.md §8d): per-pixel L-inf <= REL_TOL * max(1, |ref|) on >= MIN_FRAC of the pixels, RGBA8
    within 1 LSB on >= MIN_FRAC, mean-image relative error < 1e-3.  Prints the worst pixel."""
    s = stats(gpu, ref_recursive)
    s["frac_u8_1lsb"] = frac_u8_within(gpu, ref_recursive)
    s["worst"] = worst_pixel(gpu, ref_recursive)
    print(label, "vs recursive oracle", s)
    assert s["frac_ok"] >= MIN_FRAC, s
    assert s["frac_u8_1lsb"] >= MIN_FRAC, s
    assert s["mean_rel_err"] < 1e-3, s
    return s
