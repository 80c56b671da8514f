"""A/B throughput of diagnostic library builds: python tools/probes/gpu_ab.py libA.so libB.so ...
Each build runs in its own process (HSIM_LIB), interleaved twice; prints env steps/s at 4096 envs."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CODE = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); from gpu_probe import throughput; "
        "throughput(4096, 300)") % (ROOT, os.path.join(ROOT, "tools", "probes"))

if __name__ == "__main__":
    libs = sys.argv[1:]
    for rep in range(int(os.environ.get("AB_REPS", 2))):
        for lib in libs:
            env = dict(os.environ, HSIM_LIB=os.path.abspath(lib))
            out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=120)
            line = [ln for ln in out.stdout.splitlines() if "env-steps/s" in ln]
            print(f"{os.path.basename(lib):24s} {line[-1] if line else out.stderr[-300:]}", flush=True)
