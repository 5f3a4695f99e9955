set -o pipefail
cd $GRAFT_REPO_ROOT
for a in 0 1 2 3 4 7 8; do
  echo -n "abl=$a "; CAAMD_FA64_ABL=$a timeout -k 10 120 python -u tools/bench_attn.py || exit 1
done
