set -o pipefail
cd $GRAFT_REPO_ROOT
for so in liboi.so liboi_noexp.so; do
  echo "== $so"; OI_LIB=$PWD/optimalinterpolation_amd/$so timeout -k 10 300 python scripts/lauum_probe.py 2>&1 | grep -v amdgpu.ids
done
