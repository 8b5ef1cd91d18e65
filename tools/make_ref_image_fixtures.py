"""Copies the reference's own CPU-path renders (info/images_cpu_comparison/{walled,biplane,spaceship_r1}.png,
README.md:177-194: the CPU renderer run for as long as the GPU took) into
tests/golden/ref_cpu_images.npz as RGB u8 arrays, exactly as stored (the PNG writer's flipped
orientation).  They are outputs of the reference itself, used as a statistical anchor of the
whole path (tests/test_gpu_ref_images.py): same scene and estimator, different RNG.
Run in the build container (the GPU box has no /root/reference)."""
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/info/images_cpu_comparison"


def main():
    out = {}
    for name in ("walled", "biplane", "spaceship_r1"):
        im = Image.open(os.path.join(SRC, name + ".png")).convert("RGB")
        out[name] = np.asarray(im, dtype=np.uint8)
        print(name, out[name].shape)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "ref_cpu_images.npz"), **out)


if __name__ == "__main__":
    sys.exit(main())
