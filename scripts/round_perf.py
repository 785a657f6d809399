import sys, json
sys.path.insert(0, '.')
import numpy as np
import bench
from optimalinterpolation_amd import _lib, synthetic
day = synthetic.make_day(seed=0)
perm = np.random.default_rng(99).permutation(day.ncell)
shard = day.subset(np.sort(perm[0::8]))
x0 = np.array([np.log(25e3), np.log(25e3), 0.0, 0.0, 0.0, np.log(.1)])
_lib.profile_reset()
out, st, info = _lib.gpr_batch(shard.xyt, shard.z, shard.offs, shard.xs, shard.mean, x0=x0, opt=True, info=True, profile=True)
pj = _lib.profile_json()
R = np.array(pj['rounds_log'])
print('rounds', len(R), 'total GPU ms', R[:, 4].sum(), 'wall', pj['wall_s'])
print('kernels', {k: round(v['total_ms']) for k, v in pj['kernels'].items()})
cum = np.cumsum(R[:, 4])
for q in [0, 10, 25, 50, 75, 100, 125, 150, 175, 200, len(R) - 1]:
    if q < len(R):
        print(f"round {q:4d}: eval {int(R[q,0]):5d} pred {int(R[q,1]):4d} maxT {int(R[q,2]):3d} work {R[q,3]:.3g} ms {R[q,4]:8.2f} cum {cum[q]/1e3:7.2f}s  rate {R[q,3]/R[q,4]:.3g}")
# time spent in rounds with < 256 eval cells
small = R[:, 0] < 256
print('rounds with <256 eval cells:', small.sum(), 'time', R[small, 4].sum() / 1e3, 's')
np.save('gpurun_out/rounds.npy', R)
