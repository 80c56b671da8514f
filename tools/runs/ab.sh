# A/B of the headline window (configs[1], fp64, staggered episode phases) between the default library and
# variant builds, alternating on one box, three rounds; each variant is a libhsim_<name>.so built beside
# mujocoposelearning_amd/libhsim.so (the A/B macros are listed in profiles/LOG.md), run through HSIM_LIB.
#   gpurun -- 'bash tools/runs/ab.sh r6o rsq ldle'       -> gpurun_out/r6o/ab_<name>_<round>.log
# A variant env:NAME=VALUE runs the default library with that environment variable set instead;
# BENCH_ARGS replaces the bench flags (default: the sim-only headline window).
# An optional PARITY=1 also runs the parity and reward tests on every library variant.
TAG=${1:?usage: ab.sh TAG VARIANT...}
shift
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
L=$GRAFT_REPO_ROOT/mujocoposelearning_amd
for v in "$@"; do
  case $v in env:*) ;; *) [ -f $L/libhsim_$v.so ] || { echo "missing libhsim_$v.so"; exit 2; } ;; esac
done
B="python bench.py ${BENCH_ARGS:---steps 50 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin}"
name() { case $1 in env:*) echo $1 | sed 's/^env://; s/[^A-Za-z0-9]/_/g' ;; *) echo $1 ;; esac; }
for i in 1 2 3; do
  timeout -k 10 300 $B > $O/ab_def_$i.log 2>&1 || exit 3
  for v in "$@"; do
    case $v in
      env:*) env ${v#env:} timeout -k 10 300 $B > $O/ab_$(name $v)_$i.log 2>&1 || exit 4 ;;
      *) HSIM_LIB=$L/libhsim_$v.so timeout -k 10 300 $B > $O/ab_${v}_$i.log 2>&1 || exit 4 ;;
    esac
  done
done
if [ "$PARITY" = 1 ]; then
  for v in "$@"; do
    case $v in env:*) continue ;; esac
    HSIM_LIB=$L/libhsim_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reward_eval.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests_$v.log 2>&1
    rc=$?
    echo "rc $rc" >> $O/tests_$v.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 5; fi
  done
fi
grep -o '"ms_per_step": [0-9.]*' $O/ab_*.log
