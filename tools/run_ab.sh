set -o pipefail
# A/B of the headline bench: the default libmgs_gpu.so against the variants
# named on the command line (libmgs_gpu_<v>.so), after the GPU suite on the
# default build.  Usage: bash tools/run_ab.sh v1 [v2 ...]
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -15 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in a b c; do for v in base "$@"; do
  if [ $v = base ]; then L=""; else L=libmgs_gpu_$v.so; fi
  MGS_LIB_MAIN=$L timeout -k 10 100 python bench.py --cpu-budget 0 --e2e-steps 0 > $O/$v.$r.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); print('$v.$r', round(d['value']))"
done; done
