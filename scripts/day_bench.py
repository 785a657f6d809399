"""Timing of the day pipeline's device steps on a
full-size synthetic 25 km day (~1e4 ice cells, ~53k training points):
neighbour query + gather (oi_ball_query, oi_gather_rows), the five
smoothings (oi_smooth_fields) and pass 2 (oi_gpr_batch opt=False over every
cell).  Pass 1 is replaced by fixed smooth hyper fields (its cost is the
main bench).  CPU comparison: scipy cKDTree queries and the oracle's
smoothing on the host, single thread.

Usage: python scripts/day_bench.py [--reps 3] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--out', default='')
    ap.add_argument('--no-cpu', action='store_true')
    a = ap.parse_args()
    import torch
    from optimalinterpolation_amd import day, synthetic
    d = synthetic.make_binned_day(seed=0)
    ids = np.where(~np.isnan(d.sie))
    X = np.array([d.x[ids], d.y[ids]]).T
    u = np.sin(X[:, 0] / 3e5) * np.cos(X[:, 1] / 4e5)
    rows = np.column_stack([0.3 + 0.01 * u, 0.02 + 0.001 * u, -100 + u, 2.5e5 * (1.1 + u),
                            3.0e5 * (1.1 - 0.5 * u), 6.0 + 2 * u, 4e-3 * (1.2 + u),
                            8e-4 * (1.2 - 0.5 * u)])
    out = {'ncell': int(len(X))}
    for mode in ('device', 'kdtree'):
        day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, pass1_rows=rows, neighbours=mode)  # warm
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, pass1_rows=rows, neighbours=mode)
            ts.append((time.perf_counter() - t0, res.info['timing']))
        best = min(ts, key=lambda x: x[0])
        out[mode] = {'wall_s': best[0], 'timing': best[1], 'n_train': res.info['n_train'],
                     'obs_per_cell_mean': float(np.mean(res.info['counts'])),
                     'pass2_cells_per_s': len(X) / best[1]['pass2_s']}
        print(mode, json.dumps(out[mode]), flush=True)
    if not a.no_cpu:
        from scipy.spatial import cKDTree
        from oracle import day_oracle as D
        xt, yt, _, _ = D.training_set(d.sat, d.x, d.y)
        t0 = time.perf_counter()
        tree = cKDTree(np.column_stack([xt, yt]))
        for q in X:
            tree.query_ball_point(x=q, r=300e3)
        t_kd = time.perf_counter() - t0
        g = np.zeros(d.sie.shape) * np.nan
        g[ids] = rows[:, 3]
        t0 = time.perf_counter()
        D.smooth(g, 6e5, d.sie, 2)
        t_sm = (time.perf_counter() - t0) * 5
        out['cpu'] = {'ckdtree_query_all_s': t_kd, 'oracle_smooth_5_fields_s': t_sm, 'cores': 1}
        print('cpu', json.dumps(out['cpu']), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
