# round 5: eigensolver tridiagonalisation width (OI_SY_S) and the round-4
# pending eigensolver (branch eigh-opt-pending) on the probe; config-2 test
set -o pipefail
D=gpurun_out/r05/b; mkdir -p $D
for s in 8 16 32; do
  OI_SY_S=$s timeout -k 10 120 tools/eigh_probe 928 32 > $D/eigh_probe_s$s.txt 2>&1 || { cat $D/eigh_probe_s$s.txt; exit 1; }
  echo "S=$s: $(head -1 $D/eigh_probe_s$s.txt)"
done
timeout -k 10 120 tools/eigh_probe_pend 928 32 > $D/eigh_probe_pend.txt 2>&1 || { cat $D/eigh_probe_pend.txt; exit 1; }
echo "pend: $(head -1 $D/eigh_probe_pend.txt)"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_config2.py -x -v -s --timeout 200 --timeout-method thread > $D/config2.log 2>&1
rc=$?; grep -E "config 2 T1|PASSED|FAILED|passed|failed" $D/config2.log | tail -4; exit $rc
