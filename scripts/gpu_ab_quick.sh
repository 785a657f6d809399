# quick A/B on fixed cells (scripts/lauum_probe.py) for several builds, 2 reps
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for so in "$@"; do
  echo "== $so"; OI_LIB=$PWD/optimalinterpolation_amd/$so timeout -k 10 300 python scripts/lauum_probe.py 2>&1 | grep -v amdgpu.ids
done; done
