"""Is a random-init Mixtral's greedy output stable under bf16-sized perturbations?

For depth L in DEPTHS (Mixtral-8x7B width, L layers), 8 fixed prompts:
  * engine:  the bf16 EP = 1 engine's first 2 greedy tokens vs the fp32 dense oracle
             (bench_tp._dense_agreement: rank / gap of each engine token under the oracle);
  * flip:    a second fp32 oracle whose MoE input is rounded to bf16 before routing (a 2^-9
             relative perturbation, what any bf16 engine does), teacher-forced on the same
             prompts: how many (token, layer) top-2 selections change, and the rank of the
             perturbed oracle's argmax under the unperturbed one.
If the perturbed fp32 oracle disagrees with the fp32 oracle as much as the engine does, the
disagreement is the model's routing sensitivity, not the kernels.

Usage (GPU): DEPTHS=2,8,32 python scripts/ep_chaos_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mlopamd.models import build_model  # noqa: E402
from mlopamd.models import reference as R  # noqa: E402
from mlopamd.models.config import get_config  # noqa: E402
from mlopamd.runtime.bench_tp import PROMPTS, _clamp_prompts, _dense_agreement  # noqa: E402
from mlopamd.runtime.engine import Engine, EngineConfig  # noqa: E402
from mlopamd.runtime.sampler import SamplingParams  # noqa: E402

_orig_mlp = R._mlp
STATS = {"sel": 0, "flips": 0}


def _rounded_mlp(model, i, x):
    xr = x.to(torch.bfloat16).float()
    L = model.layers[i]
    a = torch.topk(torch.nn.functional.linear(x, L["router"].float()), model.cfg.top_k, -1).indices.sort(-1).values
    b = torch.topk(torch.nn.functional.linear(xr, L["router"].float()), model.cfg.top_k, -1).indices.sort(-1).values
    STATS["sel"] += a.shape[0]
    STATS["flips"] += int((a != b).any(-1).sum())
    return _orig_mlp(model, i, xr)


def main():
    dev = torch.device("cuda:0")
    name = os.environ.get("MODEL", "mixtral-8x7b")
    out = []
    for depth in [int(x) for x in os.environ.get("DEPTHS", "2,8,32").split(",")]:
        cfg = get_config(name, num_layers=depth)
        model = build_model(cfg, device=dev, dtype=torch.bfloat16, seed=7)
        prompts = _clamp_prompts(PROMPTS, cfg.vocab_size)
        eng = Engine(model, EngineConfig(max_num_seqs=8, max_num_batched_tokens=1024, max_model_len=256,
                                         num_kv_blocks=80, use_graphs=False, async_scheduling=False))
        toks = eng.generate(prompts, SamplingParams(max_tokens=2, ignore_eos=True))
        eng.shutdown()
        row = {"model": name, "layers": depth, "engine": _dense_agreement(model, prompts, toks)}
        ranks = []
        STATS.update(sel=0, flips=0)
        for p in prompts:
            base = R.dense_logits(model, p)[-1]
            R._mlp = _rounded_mlp
            try:
                pert = R.dense_logits(model, p)[-1]
            finally:
                R._mlp = _orig_mlp
            ranks.append(int((base > base[int(pert.argmax())]).sum()))
        row["flip"] = {"router_selections": STATS["sel"], "changed": STATS["flips"],
                       "perturbed_argmax_rank": ranks}
        print(json.dumps(row), flush=True)
        out.append(row)
        del model
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/ep_chaos.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
