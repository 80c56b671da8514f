# round 4 m: diagnosis of the README-config learning curve (r4l: ep_rew_mean 46-48 at 20 M on 3 seeds,
# log_std rising linearly 0 -> 2.3).  Causal checks, stand, fp64, staggered clocks:
#  (a, b) README config with ent_coef 0 (seeds 0, 1), 20 M steps
#  (c) the reference's config.py hyperparameters (README.md:154), seed 0, 20 M steps
#  (d) README config in the literal layout (8 envs x 2048 steps), seed 0, 3 M steps
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4m
P=tools/probes/gpu_learning_curve_ref.py
timeout -k 10 1120 python -u $P --seed 0 --steps 20e6 --every 10 --stagger --ent-coef 0 > gpurun_out/r4m/lc_ent0_seed0.log 2>&1 &
p1=$!
timeout -k 10 1120 python -u $P --seed 1 --steps 20e6 --every 10 --stagger --ent-coef 0 > gpurun_out/r4m/lc_ent0_seed1.log 2>&1 &
p2=$!
timeout -k 10 1120 python -u $P --seed 0 --steps 20e6 --every 10 --stagger --config configpy > gpurun_out/r4m/lc_cfg_seed0.log 2>&1 &
p3=$!
timeout -k 10 1120 python -u $P --seed 0 --steps 3e6 --every 2 --envs 8 --n-steps 2048 --stagger > gpurun_out/r4m/lc_literal_seed0.log 2>&1 &
p4=$!
rc=0
for p in $p1 $p2 $p3 $p4; do wait $p || rc=$?; done
exit $rc
