"""HF checkpoints served on the MI355X: tiny Llama / Mixtral models saved by transformers,
loaded (bf16) into the GPU engine (HIP kernels, hipGraph decode, lazy KV arena); every
greedy token the engine emits is transformers' fp32 argmax up to bf16 ties."""
import pytest
import torch

from mlopamd.models import loader
from mlopamd.runtime.engine import Engine, EngineConfig
from mlopamd.runtime.sampler import SamplingParams

pytestmark = pytest.mark.gpu
transformers = pytest.importorskip("transformers")


def _save(tmp_path, family):
    kw = dict(vocab_size=512, hidden_size=256, num_hidden_layers=2, num_attention_heads=2, num_key_value_heads=1,
              head_dim=128, max_position_embeddings=512)
    torch.manual_seed(3)
    if family == "mixtral":
        m = transformers.MixtralForCausalLM(transformers.MixtralConfig(intermediate_size=256, num_local_experts=4,
                                                                       num_experts_per_tok=2, **kw))
    else:
        m = transformers.LlamaForCausalLM(transformers.LlamaConfig(
            intermediate_size=512, rope_parameters={"rope_theta": 500000.0, "rope_type": "default"}, **kw))
    m = m.eval()
    m.save_pretrained(tmp_path)
    return m


@pytest.mark.parametrize("family", ["llama", "mixtral"])
def test_hf_checkpoint_on_gpu_engine(gpu, tmp_path, family):
    hf = _save(tmp_path, family)
    model = loader.load_pretrained(tmp_path, device=gpu)
    eng = Engine(model, EngineConfig(max_num_seqs=4, max_num_batched_tokens=64, max_model_len=256,
                                     num_kv_blocks=64, graph_buckets=(1, 2, 4)))
    g = torch.Generator().manual_seed(11)
    prompts = [torch.randint(3, 500, (n,), generator=g).tolist() for n in (41, 7, 90)]
    outs = eng.generate(prompts, SamplingParams(max_tokens=8, ignore_eos=True))
    assert eng.stats["graph_steps"] > 0
    for p, o in zip(prompts, outs):
        seq = p + o
        with torch.no_grad():
            lg = hf(torch.tensor([seq])).logits[0].float()
        for j, tok in enumerate(o):
            row = lg[len(p) - 1 + j]
            assert row[tok] >= row.max() - 0.05 * row.abs().max(), (family, j, tok, int(row.argmax()))
