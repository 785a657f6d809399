"""Regenerate profiles/pmc_traffic.json (the `roofline.traffic` bench.py
reports) from a pmc_summary.py output of the driver's command: HBM bytes per
dispatch per kernel, under the names the library's profile uses
(k_lauum_grad1 -> k_lauum_grad, every k_chol_panel<...> / k_panel_even<...>
instantiation -> k_chol_panel / k_panel_even, dispatch-weighted;
k_diag_factor4w -> k_diag_factor).  Kernels measured in
earlier rounds and absent from this pass (k_svgp_train) keep their entries.
Usage: python scripts/r06/pmc_traffic.py profiles/r06/final/pmc_hbm_summary.json"""
import json
import sys

ALIAS = {'k_lauum_grad1': 'k_lauum_grad', 'void k_chol_panel<false>': 'k_chol_panel',
         'void k_chol_panel<true>': 'k_chol_panel', 'k_diag_factor4w': 'k_diag_factor'}


def main(path, out='profiles/pmc_traffic.json'):
    summ = json.load(open(path))['kernels']
    old = json.load(open(out))
    new = {'_source': (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel trace only) of "
                       f"python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline on "
                       f"the round-6 tree (scripts/r06/gpu_prof.sh); FETCH_SIZE x2 (gfx950), KB -> bytes; {path}")}
    acc = {}
    for k, v in summ.items():
        name = ALIAS.get(k, k)
        for tmpl in ('k_chol_panel', 'k_panel_even'):  # template instantiations
            if name.startswith(f'void {tmpl}<'):
                name = tmpl
        a = acc.setdefault(name, [0, 0.0, 0.0])
        a[0] += v['dispatches']
        a[1] += v['fetch_bytes_per_dispatch'] * v['dispatches']
        a[2] += v['write_bytes_per_dispatch'] * v['dispatches']
    for name, (nd, fb, wb) in acc.items():
        nd = max(nd, 1)
        new[name] = {'dispatches': nd, 'fetch_bytes_per_launch': fb / nd, 'write_bytes_per_launch': wb / nd,
                     'hbm_bytes_per_launch': (fb + wb) / nd}
    if 'k_lauum_grad' in new:
        new['k_lauum_grad1'] = new['k_lauum_grad']
    for k, v in old.items():  # measured in earlier rounds only (other workloads)
        if k == 'k_svgp_train' and k not in new:
            new[k] = v
    json.dump(new, open(out, 'w'), indent=1)


if __name__ == '__main__':
    main(*sys.argv[1:])
