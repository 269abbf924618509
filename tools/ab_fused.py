"""A/B timing of the fused minibatch gradient (fused_update_kernel + slab reduction) between two
builds of the package, alternated in one process pair per round to cancel clock drift.

usage: python tools/ab_fused.py ROOT_A ROOT_B [rounds]   (each ROOT holds a built package)
Runs each build in its own subprocess (one library per process), R rounds of 50 timed calls,
and prints the per-call microseconds of each round and the medians."""
import json
import os
import subprocess
import sys

CHILD = r'''
import sys, json, torch
sys.path.insert(0, sys.argv[1])
from mujoco_reinforcement_learning_amd.agent import PPOEngineAgent
from mujoco_reinforcement_learning_amd.runconfig import make_run
from mujoco_reinforcement_learning_amd import engine as E
dev = torch.device("cuda", 0)
b, n, t = 65536, 4096, 128
run = make_run(hidden=(256, 256), rng="philox", precision="bf16")
torch.manual_seed(0)
agent = PPOEngineAgent(run, device=dev)
g = torch.Generator(device=dev).manual_seed(0)
st = torch.randn(n * t, 17, device=dev, generator=g)
ac = torch.randn(n * t, 6, device=dev, generator=g)
lp = torch.randn(n * t, device=dev, generator=g) - 5
ad = torch.randn(n * t, device=dev, generator=g)
vt = torch.randn(n * t, device=dev, generator=g)
rows = torch.empty(b, dtype=torch.int32, device=dev)
loss = torch.empty(2, device=dev)
eng = agent.engine
eng.stage_records(st, ac, lp, ad, vt)
E.feistel_rows(1, 0, 0, b, n, t, rows)
def call(k):
    eng.minibatch_grad_staged(rows, b, agent.flat_grad, loss, 0.9, 1.1, 1e-4, 1 / b, 1 / (b * 6),
                              weights_current=k > 0)
for k in range(10):
    call(k)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for k in range(50):
    call(1)
e1.record()
torch.cuda.synchronize()
eng.timing(True, capacity=4096)
for k in range(50):
    call(1)
torch.cuda.synchronize()
ks = {n: 1000 * r["ms"] / r["launches"] for n, r in eng.timing_kernels().items()}
eng.timing(False)
print(json.dumps({"us": 1000 * e0.elapsed_time(e1) / 50, "kernels_us": ks}))
'''


def main():
    a, b = sys.argv[1], sys.argv[2]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    res = {"A": [], "B": []}
    for r in range(rounds):
        for tag, root in (("A", a), ("B", b)):
            out = subprocess.run([sys.executable, "-c", CHILD, root], capture_output=True,
                                 text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:])
                raise SystemExit(f"{tag} failed")
            rec = json.loads(out.stdout.strip().splitlines()[-1])
            us = rec["us"]
            res[tag].append(us)
            kus = ", ".join(f"{k} {v:.2f}" for k, v in sorted(rec["kernels_us"].items()))
            print(f"round {r} {tag}: {us:.2f} us per fused minibatch gradient ({kus})", flush=True)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print(json.dumps({"median_us": med, "rounds": res}))


if __name__ == "__main__":
    main()
