"""Dump the PPO update's epoch HIP graph (world 1: every minibatch step of an epoch as one graph) as
a DOT file and count its node kinds, to see what sits between the kernels that rocprofv3's kernel
trace shows idle gaps around.   python tools/probes/gpu_graph_dump.py OUT_DIR"""
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

_Orig = torch.cuda.CUDAGraph


class _DebugGraph(_Orig):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.enable_debug_mode()


torch.cuda.CUDAGraph = _DebugGraph

from mujocoposelearning_amd import ppo as P  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/graph_dump"
    os.makedirs(out, exist_ok=True)
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}},
                         n_envs=4096, model=HsModel(XML), seed=0, precision="fp64")
    ppo = P.PPO(env, n_steps=32, batch_size=32768, n_epochs=1, learning_rate=3e-4, seed=0,
                policy_kwargs={"net_arch": {"pi": [256, 256], "vf": [256, 256]}, "activation_fn": "ReLU"})
    adv, ret = ppo.collect_rollouts()
    ppo.train(adv, ret)
    torch.cuda.synchronize()
    ge = getattr(ppo, "_epoch_graph", None)
    if ge is None:
        print("no epoch graph")
        return
    path = os.path.join(out, "epoch_graph.dot")
    try:
        ge.debug_dump(path)
        text = open(path).read()
    except (RuntimeError, OSError) as e:   # the DOT dump is not available on every runtime
        print("no DOT dump:", e)
        text = ""
    kinds = collections.Counter(re.findall(r'(KERNEL|MEMSET|MEMCPY|EVENT_RECORD|WAIT_EVENT|EMPTY|HOST|GRAPH|'
                                           r'MEM_ALLOC|MEM_FREE)', text))
    print("node kinds:", dict(kinds))
    print("dot bytes:", len(text))
    # host cost of a replay against its GPU time: is the update's graph replay submission-bound?
    import time
    perm = torch.randperm(ppo.n_steps * env.num_envs, device="cuda")
    ppo._g_perm.copy_(perm)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        ge.replay()
    torch.cuda.synchronize()
    ev0.record()
    t0 = time.perf_counter()
    for _ in range(5):
        ge.replay()
    t1 = time.perf_counter()
    ev1.record()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"5 epoch replays: host submit {1e3 * (t1 - t0):.2f} ms, GPU {ev0.elapsed_time(ev1):.2f} ms, "
          f"wall {1e3 * (t2 - t0):.2f} ms; kernels per replay {kinds.get('KERNEL', 0)}")
    env.close()


if __name__ == "__main__":
    main()
