"""HF checkpoint loading (models/loader.py) against an INDEPENDENT implementation:
tiny Llama / Mixtral models built and saved by Hugging Face ``transformers`` (random
init, safetensors), loaded into our layout, must reproduce transformers' own logits
(fp32, CPU) through our dense oracle AND generate the same greedy tokens through the
serving engine (paged KV, chunked prefill, continuous batching).  This pins the weight
mapping (fused QKV, 16-row gate/up interleave, expert stacking) and the math conventions
(rotate-half RoPE with rope_parameters.rope_theta, GQA, RMSNorm, SiLU, top-2 routing)."""
import json

import pytest
import torch

from mlopamd.models import loader
from mlopamd.models.reference import dense_logits
from mlopamd.runtime.engine import Engine, EngineConfig
from mlopamd.runtime.sampler import SamplingParams

transformers = pytest.importorskip("transformers")


def _tiny_llama(tmp_path, tie=False):
    cfg = transformers.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                   num_attention_heads=2, num_key_value_heads=1, head_dim=128,
                                   max_position_embeddings=512, rms_norm_eps=1e-5, tie_word_embeddings=tie,
                                   rope_parameters={"rope_theta": 500000.0, "rope_type": "default"})
    torch.manual_seed(0)
    m = transformers.LlamaForCausalLM(cfg).eval()
    with torch.no_grad():  # non-trivial norm weights: a swapped norm would show
        for n, p in m.named_parameters():
            if n.endswith("layernorm.weight") or n == "model.norm.weight":
                p.copy_(1 + 0.2 * torch.randn_like(p))
    m.save_pretrained(tmp_path)
    return m


def _tiny_mixtral(tmp_path):
    cfg = transformers.MixtralConfig(vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2,
                                     num_attention_heads=2, num_key_value_heads=1, head_dim=128,
                                     num_local_experts=4, num_experts_per_tok=2, max_position_embeddings=512)
    torch.manual_seed(1)
    m = transformers.MixtralForCausalLM(cfg).eval()
    m.save_pretrained(tmp_path)
    return m


def _hf_greedy(m, prompt, n):
    out = m.generate(torch.tensor([prompt]), max_new_tokens=n, do_sample=False, min_new_tokens=n,
                     pad_token_id=0, eos_token_id=None)
    return out[0, len(prompt):].tolist()


@pytest.mark.parametrize("family", ["llama", "llama_tied", "mixtral"])
def test_hf_checkpoint_parity(tmp_path, family):
    hf = _tiny_mixtral(tmp_path) if family == "mixtral" else _tiny_llama(tmp_path, tie=family == "llama_tied")
    cfg = loader.config_from_hf(json.loads((tmp_path / "config.json").read_text()))
    assert cfg.rope_theta == (1e6 if family == "mixtral" else 5e5) and cfg.is_moe == (family == "mixtral")
    ours = loader.load_pretrained(tmp_path, device="cpu", dtype=torch.float32)
    toks = torch.randint(3, 500, (37,), generator=torch.Generator().manual_seed(5)).tolist()
    with torch.no_grad():
        ref = hf(torch.tensor([toks])).logits[0].float()
    got = dense_logits(ours, toks)
    torch.testing.assert_close(got, ref, atol=2e-4, rtol=1e-3)
    # the serving engine on the loaded weights generates transformers' greedy continuation
    eng = Engine(ours, EngineConfig(max_num_seqs=4, max_num_batched_tokens=16, max_model_len=256,
                                    num_kv_blocks=64, use_graphs=False))
    prompts = [toks, toks[:9]]
    outs = eng.generate(prompts, SamplingParams(max_tokens=6, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert o == _hf_greedy(hf, p, 6)


def test_resolve_model_dir(tmp_path, monkeypatch):
    d = tmp_path / "1" / "abc" / "artifacts" / "model"
    d.mkdir(parents=True)
    assert loader.resolve_model_dir(str(d)) is None  # no checkpoint yet
    (d / "config.json").write_text("{}")
    (d / "model.safetensors").write_bytes(b"")
    assert loader.resolve_model_dir(str(d)) == d
    assert loader.resolve_model_dir("file://" + str(d.parent)) == d  # .../artifacts -> model/
    monkeypatch.setenv("MLOP_ARTIFACT_ROOT", str(tmp_path))
    assert loader.resolve_model_dir("s3://mlflow/1/abc/artifacts") == d  # reference URI rewrite shape
    monkeypatch.delenv("MLOP_ARTIFACT_ROOT")
    assert loader.resolve_model_dir("s3://mlflow/1/abc/artifacts") is None
    assert loader.resolve_model_dir("hf://x") is None and loader.resolve_model_dir(None) is None


def test_unsupported_architecture_is_rejected():
    with pytest.raises(ValueError, match="unsupported"):
        loader.config_from_hf({"architectures": ["GPT2LMHeadModel"], "hidden_size": 8, "num_attention_heads": 1,
                               "vocab_size": 8, "intermediate_size": 8, "num_hidden_layers": 1})


def _word_tokenizer(path):
    from tokenizers import Tokenizer, models, pre_tokenizers

    vocab = {w: i for i, w in enumerate(["[UNK]", "<s>", "</s>"] + [f"w{i}" for i in range(200)] +
                                          ["hello", "world", "mi355x"])}
    tok = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    tok.save(str(path / "tokenizer.json"))
    return tok


def test_operator_deploys_hf_checkpoint_end_to_end(tmp_path):
    """MLflow version whose artifact is an HF checkpoint (+ tokenizer.json) -> MlflowModel CR
    -> SeldonDeployment -> a real predictor PROCESS (V2 server on CPU) serving those weights:
    /generate on text returns transformers' greedy continuation, decoded by the checkpoint's
    own tokenizer."""
    import asyncio

    import aiohttp

    from mlopamd.controller import seldon
    from mlopamd.controller.app import make_operator
    from mlopamd.controller.clock import RealClock
    from mlopamd.controller.crd import GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION, \
        OperatorSettings
    from mlopamd.controller.kube import FakeKube
    from mlopamd.controller.local import FakeSeldonController, ProcessLauncher, mlflow_model_cr, wait_for
    from mlopamd.controller.mlflow import LocalMlflowClient, SqliteRegistry
    from mlopamd.controller.prometheus import LocalProm, MetricStore

    ck = tmp_path / "1" / "run" / "artifacts" / "model"
    ck.mkdir(parents=True)
    hf = _tiny_llama(ck)
    tok = _word_tokenizer(ck)
    prompt = "hello world w7 w42 mi355x w3"
    ids = tok.encode(prompt).ids
    expect = _hf_greedy(hf, ids, 5)

    async def go():
        kube, reg = FakeKube(), SqliteRegistry()
        reg.create_model_version("tiny", f"file://{ck.parent}", tags={"mlop.runtime": seldon.RUNTIME_LLM})
        reg.set_alias("tiny", "champion", 1)
        op, _ = make_operator(kube, LocalMlflowClient(reg), LocalProm(MetricStore()), RealClock(), OperatorSettings())
        launcher = ProcessLauncher(ready_timeout_s=240, extra_env={
            "MLOP_DEVICE": "cpu", "MLOP_DTYPE": "float32", "MLOP_ENGINE_USE_GRAPHS": "false",
            "MLOP_ENGINE_NUM_KV_BLOCKS": "64", "MLOP_ENGINE_MAX_MODEL_LEN": "256", "OMP_NUM_THREADS": "2"})
        ctl = FakeSeldonController(kube, launcher, RealClock()).start()
        await op.start()
        try:
            await kube.create(GROUP, VERSION, "ns", PLURAL, mlflow_model_cr("tiny", "ns", "tiny", "champion"))

            async def ready():
                o = await kube.get(GROUP, VERSION, "ns", PLURAL, "tiny")
                return (o.get("status") or {}).get("ready") == "True"

            await wait_for(ready, 240)
            sd = await kube.get(SELDON_GROUP, SELDON_VERSION, "ns", SELDON_PLURAL, "tiny")
            assert sd["spec"]["predictors"][0]["graph"]["modelUri"] == f"file://{ck.parent}"
            pod = next(iter(ctl.pods.values()))
            async with aiohttp.ClientSession() as s:
                async with s.post(pod.endpoint + "/v2/models/tiny/generate",
                                  json={"text_input": prompt, "parameters": {"max_tokens": 5}}) as r:
                    assert r.status == 200, await r.text()
                    body = await r.json()
            return body
        finally:
            await ctl.stop()
            await op.stop()

    body = asyncio.run(asyncio.wait_for(go(), 300))
    assert body["output_ids"] == expect
    assert body["text_output"] == tok.decode(expect, skip_special_tokens=True)


@pytest.mark.parametrize("patch,msg", [
    ({"rope_scaling": {"rope_type": "yarn", "factor": 4.0}}, "rope_scaling"),
    ({"rope_scaling": {"type": "linear", "factor": 2.0}}, "rope_scaling"),
    ({"sliding_window": 4096, "max_position_embeddings": 32768}, "sliding_window"),
    ({"attention_bias": True}, "attention_bias"),
    ({"mlp_bias": True}, "mlp_bias"),
])
def test_unservable_settings_are_rejected(patch, msg):
    base = {"architectures": ["LlamaForCausalLM"], "hidden_size": 256, "num_attention_heads": 2,
            "vocab_size": 512, "intermediate_size": 512, "num_hidden_layers": 1}
    with pytest.raises(ValueError, match=msg):
        loader.config_from_hf(dict(base, **patch))
    cfg = loader.config_from_hf(dict(base, sliding_window=None, attention_bias=False,
                                     eos_token_id=[128001, 128008, 128009]))
    assert cfg.eos_ids == (128001, 128008, 128009)
