"""Diagnostic: per-minibatch loss values of the bf16 graph-vs-eager case (tests/
test_gpu_iteration.py::test_graphs_match_eager) with the in-launch fold on / off."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from parity_util import make_pair  # noqa: E402


def run(fold, graph, iters=3):
    algo, agent, *_ = make_pair("cuda:0", n=128, t=16, b=512, epochs=2, hidden=(256, 256),
                                p_term=0.05, rng="philox", seed=4, rollout_graph=graph,
                                train_graph=graph, precision="bf16")
    agent.engine.fused_fold(fold)
    out = []
    for _ in range(iters):
        algo.iterate(verbose=False)
        torch.cuda.synchronize()
        out.append((algo._loss_buf.detach().cpu().clone(), agent.packed_params().cpu().clone()))
    return out


res = {}
for fold in (False, True):
    for graph in (False, True):
        res[(fold, graph)] = run(fold, graph)
res[("fold-again", True)] = run(True, True)
base = res[(False, False)]
for key, r in res.items():
    for it, ((lb, p), (lb0, p0)) in enumerate(zip(r, base)):
        d = (lb != lb0)
        print(f"fold={key[0]} graph={key[1]} it={it} params_equal={torch.equal(p, p0)} "
              f"loss_diff_at={d.nonzero().tolist()}")
        if d.any():
            print("   eager/no-fold:", lb0[..., 0].flatten().tolist())
            print("   this        :", lb[..., 0].flatten().tolist())
