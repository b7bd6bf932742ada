"""Same-box eager PyTorch-ROCm baseline: stock Hugging Face
``LlamaForCausalLM`` with the Llama-3-8B architecture, bf16, random-init weights,
``generate()`` (greedy, dynamic KV cache, SDPA attention, torch.matmul = hipBLASLt
GEMMs, no graphs) on a static batch of B prompts of P random tokens, O new tokens
each.  This is what a stock Python model server would run for the predictor; the
result line is comparable to bench.py's served tokens/s (generated tokens / s)."""
import json
import os
import sys
import time

import torch

B = int(os.environ.get("B", 256))
P = int(os.environ.get("P", 256))
O = int(os.environ.get("O", 256))
LAYERS = int(os.environ.get("LAYERS", 32))


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def main():
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=LAYERS,
                      num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192,
                      rms_norm_eps=1e-5, rope_theta=500000.0, tie_word_embeddings=False,
                      bos_token_id=128000, eos_token_id=128001)
    dev = torch.device(os.environ.get("DEV", "cuda"))
    t0 = time.perf_counter()
    torch.set_default_dtype(torch.bfloat16)
    with dev:
        model = LlamaForCausalLM(cfg)  # random init on the GPU
    model.eval()
    for p in model.parameters():  # keep activations finite with random weights
        p.data.normal_(0.0, 0.02) if p.dim() > 1 else p.data.fill_(1.0)
    sync(dev)
    build_s = time.perf_counter() - t0
    g = torch.Generator(device=dev).manual_seed(0)
    ids = torch.randint(1000, 127000, (B, P), device=dev, generator=g)
    kw = dict(max_new_tokens=O, min_new_tokens=O, do_sample=False, pad_token_id=0,
              attention_mask=torch.ones_like(ids))
    with torch.no_grad():
        model.generate(ids[:, :32], max_new_tokens=4, min_new_tokens=4, do_sample=False, pad_token_id=0)
        sync(dev)
        t = time.perf_counter()
        out = model.generate(ids, **kw)
        sync(dev)
        el = time.perf_counter() - t
    gen = int(out.shape[0]) * (int(out.shape[1]) - P)
    print(json.dumps(dict(baseline="hf-transformers-eager", model="Llama-3-8B", layers=LAYERS, batch=B,
                          prompt_len=P, output_len=O, generated_tokens=gen, seconds=round(el, 3),
                          served_tokens_per_sec=round(gen / el, 1), build_s=round(build_s, 2),
                          attn=model.config._attn_implementation)), flush=True)


if __name__ == "__main__":
    sys.exit(main())
