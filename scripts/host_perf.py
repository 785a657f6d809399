"""Wall-time split of one day shard (non-profile run, after a warm-up call):
setup (uploads), host blocked on round completion, and the rest (host CG
steps, admission, launch enqueue)."""
import sys, time
sys.path.insert(0, '.')
import numpy as np
from optimalinterpolation_amd import _lib, synthetic
day = synthetic.make_day(seed=0)
perm = np.random.default_rng(99).permutation(day.ncell)
shard = day.subset(np.sort(perm[0::8]))
small = day.subset(np.sort(perm[0::8])[:8])
x0 = np.array([np.log(25e3), np.log(25e3), 0.0, 0.0, 0.0, np.log(.1)])
_lib.gpr_batch(small.xyt, small.z, small.offs, small.xs, small.mean, x0=x0, opt=True)
_lib.profile_reset()
t0 = time.perf_counter()
_lib.gpr_batch(shard.xyt, shard.z, shard.offs, shard.xs, shard.mean, x0=x0, opt=True)
t1 = time.perf_counter()
pj = _lib.profile_json()
print(f"python wall {t1 - t0:.3f}s  engine wall {pj['wall_s']:.3f}  setup {pj['setup_s']:.3f}  "
      f"sync-wait {pj['sync_s']:.3f}  host-other {pj['wall_s'] - pj['setup_s'] - pj['sync_s']:.3f}  rounds {pj['rounds']}")
