"""Generate tests/golden/video_helpers.npz (run in the build container only).

    python tests/golden/make_video_golden.py

Imports the reference's utils.py from /root/reference (read-only; cv2 and
pytorch_msssim are absent here and stubbed, they are not used by the helpers
below) and records, on seeded inputs, the outputs of the two helpers of the
video driver that gsvc_amd/video.py restates:

* detect_outliers_mean_diff (utils.py:214-229) -- the K-frame detector;
* EarlyStopping (utils.py:188-211) -- the iteration at which training stops.

Only the resulting .npz (inputs and outputs) is committed; the tests never run
this script and the reference never reaches the GPU box.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(REPO, "tests", "golden", "video_helpers.npz")
REF = "/root/reference"


def main():
    for name in ("cv2", "pytorch_msssim"):
        mod = types.ModuleType(name)
        mod.ms_ssim = mod.ssim = lambda *a, **k: None
        sys.modules.setdefault(name, mod)
    sys.path.insert(0, REF)
    import utils as ref_utils  # the reference's utils.py

    rng = np.random.default_rng(2025)
    rec = {}
    # K-frame detector on normalised loss lists like train_video_Represent.py:335-348
    for case in range(6):
        n = int(rng.integers(5, 120))
        vals = rng.random(n) * 0.2
        cuts = rng.choice(np.arange(1, n), size=min(n - 1, int(rng.integers(0, 6))), replace=False)
        vals[cuts] += rng.uniform(0.5, 1.0, len(cuts))
        vals[0] = 0.0
        rest = vals[1:]
        norm = np.array([vals[0]] + [(v - rest.min()) / (rest.max() - rest.min()) for v in rest])
        rec[f"outliers_in_{case}"] = norm
        rec[f"outliers_out_{case}"] = np.array(ref_utils.detect_outliers_mean_diff(list(norm)),
                                               np.int64)
    # early stopping on noisy decreasing loss curves
    for case in range(4):
        n = 3000
        curve = np.exp(-np.linspace(0, 6 + case, n)) + rng.normal(0, 1e-3 * (case + 1), n)
        es = ref_utils.EarlyStopping(patience=100, min_delta=1e-9)
        stop = -1
        for i, v in enumerate(curve):
            if es(float(v)):
                stop = i
                break
        rec[f"early_in_{case}"] = curve
        rec[f"early_stop_{case}"] = np.array(stop, np.int64)
    np.savez_compressed(OUT, **rec)
    print(OUT, sorted(rec))


if __name__ == "__main__":
    main()
