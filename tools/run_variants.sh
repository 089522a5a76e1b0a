set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/var
mkdir -p $O
for v in integ gp wf; do
  MGS_LIB_MAIN=libmgs_gpu_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -5 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
for r in a b; do for v in base integ gp wf; do
  if [ $v = base ]; then L=""; else L=libmgs_gpu_$v.so; fi
  MGS_LIB_MAIN=$L timeout -k 10 100 python bench.py --cpu-budget 0 --e2e-steps 0 > $O/$v.$r.json 2>/dev/null || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
for v in base gp; do
  if [ $v = base ]; then L=""; else L=libmgs_gpu_$v.so; fi
  MGS_LIB_MAIN=$L timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/$O/pmc_$v -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --streams 1 --cpu-budget 0 --e2e-steps 0 --no-escalate > $GRAFT_REPO_ROOT/$O/pmc_$v.log 2>&1 || exit 1
done
