"""Print the device scan of the unit-opacity alpha cut (csrc/alpha_cut.hip):
the largest kept sigma pattern (the kernels' kSigmaCutBits), the smallest
dropped one, kept patterns with exp(-sigma) > 1, kept NaN patterns.

    python tools/alpha_cut.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsvc_amd import _lib as L  # noqa: E402

lib = L.load()
out = torch.zeros(4, dtype=torch.int32, device="cuda")
t = time.perf_counter()
assert lib.gsvc_alpha_cut_scan(out.data_ptr(), None) == 0
torch.cuda.synchronize()
dt = time.perf_counter() - t
v = [int(x) & 0xFFFFFFFF for x in out.cpu().tolist()]
f = np.array(v[:2], dtype=np.uint32).view(np.float32)
print(json.dumps(dict(kept_max=hex(v[0]), drop_min=hex(v[1]), sigma_kept_max=float(f[0]),
                      sigma_drop_min=float(f[1]), kept_over_one=v[2], kept_nan=v[3],
                      constant=hex(int(lib.gsvc_alpha_cut_bits())), scan_s=round(dt, 3))))
