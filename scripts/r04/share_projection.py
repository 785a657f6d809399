"""Config-4 projection from the 8 one-GPU share runs (scripts/r04/gpu_shares.sh):
the 8-GPU day ends when its slowest share ends, so projected cells/s = day
cells / max share time; efficiency against the 1-GPU whole-day line given as
argv[2] (a bench JSON) or the shares' own cells/s-weighted single-GPU rate."""
import glob
import json
import os
import sys

d = sys.argv[1]
lines = [json.load(open(f)) for f in sorted(glob.glob(os.path.join(d, 'share_*.json')))]
cells = sum(x['config']['cells_per_rank'] for x in lines)
tmax = max(x['timed_s'] for x in lines)
one = None
if len(sys.argv) > 2:
    one = json.load(open(sys.argv[2]))['value']
tail = [x.get('rounds', {}) for x in lines]
out = {"shares": len(lines), "cells": cells, "share_s": [x['timed_s'] for x in lines],
       "share_cells": [x['config']['cells_per_rank'] for x in lines],
       "share_cells_per_s": [x['value'] for x in lines], "max_share_s": tmax,
       "projected_8gpu_cells_per_s": round(cells / tmax, 2),
       "one_gpu_cells_per_s": one,
       "projected_speedup": round(cells / tmax / one, 3) if one else None,
       "projected_efficiency": round(cells / tmax / one / len(lines), 3) if one else None,
       "tail_rounds": tail}
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(d, 'projection.json'), 'w'), indent=1)
