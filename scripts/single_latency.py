"""Config 1 latency probe: blocking one-cell opt=True calls (n = 200) with and
without the library's per-launch HIP-event profile, and the engine's run
statistics (rounds, host time blocked on the GPU).  Run under rocprofv3
--kernel-trace for the true kernel durations and the gaps between them."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
from optimalinterpolation_amd import _lib, synthetic  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402

X0 = np.array(O.X0_PRODUCTION)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cells = [synthetic.make_cells([N], seed=700 + k) for k in range(K + 2)]
dev = [(torch.from_numpy(c.xyt).cuda(), torch.from_numpy(c.z).cuda()) for c in cells]
torch.cuda.synchronize()
res = {}
for profile in (False, True, False):
    for k in range(2):  # warm
        _lib.gpr_batch_device(dev[k][0], dev[k][1], cells[k].offs, cells[k].xs, cells[k].mean, x0=X0,
                              device=0, profile=profile)
    _lib.profile_reset()
    ts, ev = [], []
    for k in range(2, K + 2):
        t0 = time.perf_counter()
        out, st, info = _lib.gpr_batch_device(dev[k][0], dev[k][1], cells[k].offs, cells[k].xs, cells[k].mean,
                                              x0=X0, info=True, device=0, profile=profile)
        ts.append(time.perf_counter() - t0)
        ev.append(int(info[0, 3]))
    pj = _lib.profile_json()
    key = f"profile={profile}" + (" (again)" if f"profile={profile}" in res else "")
    res[key] = {"ms_per_cell": round(1e3 * float(np.mean(ts)), 3),
                "us_per_eval": round(1e6 * float(np.sum(ts)) / sum(ev), 2),
                "evals_per_cell": float(np.mean(ev)),
                "engine": {k: pj[k] for k in ('rounds', 'evals', 'wall_s', 'sync_s', 'setup_s')},
                "kernels_us_per_eval": {k: round(v['total_ms'] / sum(ev) * 1e3, 2)
                                        for k, v in pj['kernels'].items() if v['launches']} if profile else None}
print(json.dumps({"n": N, "cells": K, **res}, indent=1))
