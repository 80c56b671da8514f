"""Rollout-mode (policy forward + hs_ppo_act + env step) throughput: one 4096-env batch vs G
independent env groups, each with its own torch stream, launched round-robin without cross-group
joins (a group's policy GEMMs can run while another group's step kernel finishes its tail).
python tools/probes/gpu_rollout_groups_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.model import HsModel  # noqa: E402
from mujocoposelearning_amd.ppo import ActorCritic, ppo_act  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def run(G, n=4096, steps=60):
    model = HsModel(XML)
    cfg = {"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3}
    ng = n // G
    envs = [HumanoidVecEnv(cfg, n_envs=ng, model=model, seed=g) for g in range(G)]
    pol = ActorCritic(352, 21, (256, 256)).cuda()
    pol.pack_heads()
    ls = pol.log_std.detach()
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(G - 1)]
    bufs = []
    for e in envs:
        e.reset_tensors()
        bufs.append(dict(obs=e.batch.obs, start=torch.zeros(ng, device="cuda"),
                         act=torch.empty(ng, 21, device="cuda"), clip=torch.empty(ng, 21, device="cuda"),
                         logp=torch.empty(ng, device="cuda"), val=torch.empty(ng, device="cuda"),
                         st=torch.empty(ng, device="cuda")))
    torch.cuda.synchronize()

    def step(k):
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                b = bufs[g]
                mean, value = pol.heads(b["obs"])
                ppo_act(mean, value, ls, b["start"], g, k, False, b["act"], b["clip"], b["logp"], b["val"], b["st"])
                b["obs"] = envs[g].step_tensors(b["clip"])[0]

    with torch.no_grad():
        for k in range(10):
            step(k)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(steps):
            step(10 + k)
        for s in streams[1:]:
            torch.cuda.current_stream().wait_stream(s)
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    print(f"G={G}: {ms:.3f} ms/step -> {n / ms / 1e3:.2f} M env steps/s", flush=True)
    for e in envs:
        e.close()


if __name__ == "__main__":
    for G in (1, 2, 4, 2, 1):
        run(G)
