"""Checks MGX_GRU_GRAPH: graph-captured mission GRU gives the same loss/gradients as eager
(fp32 tolerance 1e-5 rel) and times one forward+backward of the extractor at a PPO minibatch."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "minigrid-rl_amd"))
import torch
from mgx.policy import ActorCriticPolicy

T0 = time.perf_counter()
dev = "cuda:0"
torch.manual_seed(0)
B = 65536
obs = {"image": torch.randint(0, 11, (B, 12, 7, 7), dtype=torch.uint8, device=dev),
       "direction": torch.nn.functional.one_hot(torch.randint(0, 4, (B, 4), device=dev), 4).reshape(B, 16).to(torch.uint8),
       "mission": torch.randint(0, 32, (37, 128), device=dev)[torch.randint(0, 37, (B,), device=dev)]}
act = torch.randint(0, 7, (B,), device=dev)

def run(graph):
    torch.manual_seed(1)
    pol = ActorCriticPolicy(mission_cache=True).to(dev)
    pol.features_extractor.gru_graph = graph      # (MGX_GRU_GRAPH default off; forced here)
    def step():
        v, lp, ent = pol.evaluate_actions(obs, act)
        loss = (v.square().mean() - lp.mean() - 0.01 * ent.mean())
        pol.optimizer.zero_grad(set_to_none=False)
        loss.backward()
        return loss
    loss = step(); torch.cuda.synchronize()
    print("graph=%s first step done %.1fs" % (graph, time.perf_counter() - T0), flush=True)
    g = [p.grad.clone() for p in pol.parameters()]
    for _ in range(3):
        step()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    return loss.item(), g, (time.perf_counter() - t) / 10

print("setup %.1fs" % (time.perf_counter() - T0), flush=True)
l0, g0, t0 = run(False)
l1, g1, t1 = run(True)
err = max(((a - b).abs().max() / (a.abs().max() + 1e-12)).item() for a, b in zip(g0, g1))
print("aten_gru=%s loss eager %.8f graph %.8f  max rel grad diff %.3e  ms/minibatch eager %.2f graph %.2f"
      % (os.environ.get("MGX_ATEN_GRU", "0"), l0, l1, err, t0 * 1e3, t1 * 1e3), flush=True)
assert abs(l0 - l1) <= 1e-5 * max(1.0, abs(l0)) and err < 1e-4
