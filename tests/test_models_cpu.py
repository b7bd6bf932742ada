"""Model-zoo configs on CPU: Llama-3.1 (128k context via the "llama3" RoPE frequency
scaling) next to Llama-3 / Mixtral.  Oracle for the scaled frequencies: transformers'
own ``ROPE_INIT_FUNCTIONS["llama3"]`` on the same config."""
import pytest
import torch

from mlopamd.controller.placement import plan
from mlopamd.models import build_model
from mlopamd.models.config import LLAMA3_8B, get_config
from mlopamd.models.layers import rope_inv_freq


@pytest.mark.parametrize("name", ["llama3.1-8b", "llama3.1-70b"])
def test_llama31_rope_scaling_matches_transformers(name):
    tr = pytest.importorskip("transformers")
    from transformers.modeling_rope_utils import ROPE_INIT_FUNCTIONS

    c = get_config(name)
    hf = tr.LlamaConfig(hidden_size=c.hidden_size, num_attention_heads=c.num_heads,
                        num_key_value_heads=c.num_kv_heads, max_position_embeddings=c.max_position,
                        rope_theta=c.rope_theta, rope_scaling=dict(c.rope_scaling))
    ref, scale = ROPE_INIT_FUNCTIONS["llama3"](hf, "cpu")
    ours = rope_inv_freq(c.head_dim, c.rope_theta, c.rope_scaling)
    assert scale == 1.0
    torch.testing.assert_close(ours.float(), ref.float(), rtol=1e-6, atol=1e-9)
    # same shapes as Llama-3, 16x the context
    base = get_config(name.replace("3.1", "3"))
    assert (c.hidden_size, c.num_layers, c.intermediate_size) == (base.hidden_size, base.num_layers,
                                                                   base.intermediate_size)
    assert c.max_position == 16 * base.max_position


def test_llama31_aliases_and_placement():
    assert get_config("meta-llama/Llama-3.1-8B").name == "llama3.1-8b"
    p = plan("llama3.1-8b", max_model_len=131072, max_num_seqs=16)
    assert p.fits and p.tensorParallel == 1


def test_llama31_tiny_forward_uses_scaled_table():
    """A small Llama-3.1-shaped model builds its RoPE table from the scaled frequencies."""
    c = get_config("llama3.1-8b", num_layers=1, hidden_size=256, intermediate_size=512, num_heads=2,
                   num_kv_heads=1, vocab_size=512, max_position=4096)
    m = build_model(c, device="cpu", dtype=torch.float32, seed=0)
    plain = build_model(get_config("llama3-8b", num_layers=1, hidden_size=256, intermediate_size=512, num_heads=2,
                                   num_kv_heads=1, vocab_size=512, max_position=4096),
                        device="cpu", dtype=torch.float32, seed=0)
    assert m.cos_sin.shape == plain.cos_sin.shape
    assert not torch.allclose(m.cos_sin[4000], plain.cos_sin[4000])  # low frequencies stretched 8x
    assert LLAMA3_8B.rope_scaling is None
