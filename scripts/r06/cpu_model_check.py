"""Validate bench.py's CPU-baseline fit-time model at large n.

cpu_baseline() models one oracle GPR3D(opt=True) fit (GPR_CS2S3.py:143-191,
scipy CG at :166) as  k * E * t_eval(n) + t_pred(n),  with t_eval / t_pred
fitted to single-evaluation probes and k calibrated on 16 full fits at
n = 300..600 only.  This script, run on the GPU box's HOST (no GPU use):

  1. runs cpu_baseline() itself (its probes + its 16 small fits, the same
     `workers` single-threaded-BLAS processes at once) to get k, t_eval, t_pred;
  2. times 16 full oracle fits at n = 1500, 2000, 2500, 3000 (4 seeds each),
     16 processes at once (the same contention as the probes);
  3. per fit: the model with the fit's OWN evaluation count
     (k * evals * t_eval + t_pred) and with the reference's E(n) from
     day_ref_fits.npz (what the bench line uses), residual = model / measured - 1.

Writes the JSON given by --out.  Usage:
    python scripts/r06/cpu_model_check.py --out gpurun_out/cpu_model_check.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

NS = (1500, 2000, 2500, 3000)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--reps', type=int, default=4)
    ap.add_argument('--budget-s', type=float, default=1050.0)
    a = ap.parse_args()
    t0 = time.time()
    bench.heartbeat()  # a stderr line a minute: the n = 3000 fits run for minutes in silence
    workers, desc = bench.host_cores()
    sizes = np.array(NS, float)
    base = bench.cpu_baseline(sizes, np.full(len(sizes), 100.0), workers, desc, t0 + 300)
    ce, cp = base['t_eval_coef'], base['t_pred_coef']
    t_eval = lambda n: ce[0] + ce[1] * n ** 2 + ce[2] * n ** 3
    t_pred = lambda n: cp[0] + cp[1] * n ** 2 + cp[2] * n ** 3
    # k(n) exactly as cpu_baseline forms it (round 6: small- and large-n calibration fits)
    (k_s, k_l), (n_s, n_l) = base.get('fit_time_model_k_small_large', [base['fit_time_model_k']] * 2), \
        base.get('fit_time_model_k_anchor_n', [450.0, 450.0])

    def k_of(n):
        x, xs, xl = np.log(t_eval(n)), np.log(t_eval(n_s)), np.log(t_eval(n_l))
        return k_s + (float(np.clip((x - xs) / (xl - xs), 0, 1)) if xl > xs else 0.0) * (k_l - k_s)
    k = k_s
    print(f"[check {time.time() - t0:.0f}s] model: k {k_s:.4f} (n={n_s:.0f}) .. {k_l:.4f} (n={n_l:.0f}), "
          f"probes {base['probe_s']}", flush=True)
    E, e_src, _ = bench.reference_evals_model()
    jobs = [('fit', n, 17 * n + r) for n in sorted(NS, reverse=True) for r in range(a.reps)]
    fits = bench.run_jobs(jobs, workers, t0 + a.budget_s)
    rows = []
    for f in sorted(fits, key=lambda f: (f['n'], f['seed'])):
        n = f['n']
        m_own = k_of(n) * f['evals'] * t_eval(n) + t_pred(n)
        m_ref = k_of(n) * float(E(n)) * t_eval(n) + t_pred(n)
        rows.append({"n": n, "seed": f['seed'], "fit_s": round(f['fit_s'], 2), "evals": f['evals'],
                     "model_own_evals_s": round(m_own, 2), "resid_own_evals": round(m_own / f['fit_s'] - 1, 4),
                     "E_ref": round(float(E(n)), 1), "model_E_ref_s": round(m_ref, 2),
                     "resid_E_ref": round(m_ref / f['fit_s'] - 1, 4)})
        print(json.dumps(rows[-1]), flush=True)
    own = np.array([r['resid_own_evals'] for r in rows])
    meas = np.array([r['fit_s'] for r in rows])
    out = {"host": desc, "workers": workers, "fits": rows, "k": k, "k_small_large": [k_s, k_l],
           "k_anchor_n": [n_s, n_l], "t_eval_coef": ce, "t_pred_coef": cp,
           "probe_s": base['probe_s'], "small_fit_residuals": base['fit_time_residuals'],
           "max_abs_resid_own_evals": float(np.max(np.abs(own))) if len(own) else None,
           "total_resid_own_evals": (float(np.sum([r['model_own_evals_s'] for r in rows]) / np.sum(meas) - 1)
                                     if len(rows) else None),
           "E_model": e_src, "wall_s": round(time.time() - t0, 1),
           "note": ("model = k(n) * evals * t_eval(n) + t_pred(n) (bench.cpu_baseline); resid = model / measured - 1; "
                    "fits of the oracle GPR3D(opt=True) on synthetic.make_cells([n], seed), "
                    f"{workers} single-threaded-BLAS processes at once")}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, 'w') as fh:
        json.dump(out, fh, indent=1)
    print(f"[check {time.time() - t0:.0f}s] wrote {a.out}: max |resid| {out['max_abs_resid_own_evals']}",
          flush=True)


if __name__ == '__main__':
    main()
