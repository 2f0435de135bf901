"""Long context on the GPU (VERDICT r5 missing #3 / next #5): Llama-3.1-8B layer widths (llama3 RoPE scaling, 128K
positions) served through the engine - chunked prefill of a 32K-token prompt, then decode - checked against the
fp32 PyTorch oracle (LlamaModel.reference_logits_at: query-chunked causal attention, no [T, T] matrix) at the last
prompt position and every decoded position.

The reference serves max-model-len 131072
(/root/reference/community/chat-llama-nemotron/backend-dynamo/config/agg_llama_nemotron_4b.yaml:21); two layers keep
the fp32 oracle cheap while every kernel runs at the full context: the prefill attention over 32K keys across 4
chunks, the split-KV decode attention at ctx > 32K, and RoPE at positions past the original 8K window.
"""
import pytest
import torch

from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,chunk", [(32768, 8192), (20000, 16384)])
def test_long_prompt_prefill_decode_matches_fp32(cuda, T, chunk):
    cfg = LlamaConfig.llama31_8b(num_layers=2)
    tok = llama3_byte_tokenizer(cfg.vocab_size)
    m = LlamaModel(cfg, device=cuda).random_init(11)
    g = torch.Generator().manual_seed(T)
    prompt = torch.randint(1000, 120000, (T,), generator=g).tolist()
    steps = 4
    eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=4, max_batched_tokens=chunk, prefill_chunk=chunk,
                                         max_model_len=T + 64, use_graphs=False, decode_steps=1, prefix_cache=False,
                                         kv_memory_fraction=0.05))
    seen = []
    fwd = m.forward

    def rec(fb, kv, ws=None):
        out = fwd(fb, kv, ws)
        if fb.sample_rows is None or fb.sample_rows.numel():
            seen.append(out.float().cpu())
        return out

    m.forward = rec
    try:
        req = eng.generate([prompt], SamplingParams(temperature=0.0, max_tokens=steps, ignore_eos=True))[0]
    finally:
        del m.forward
    out = req.output_ids
    assert len(out) == steps
    # one sampled row per forward: the last prefill chunk's final row, then one per decode step
    got = torch.cat([s for s in seen if s.shape[0] == 1])[-steps:]
    assert got.shape[0] == steps
    eng.close()
    rows = [T - 1 + i for i in range(steps)]
    ref = m.reference_logits_at(torch.tensor(prompt + out[:-1]), rows, device=cuda)
    scale = ref.abs().max().item()
    err = (got[:, : ref.shape[1]] - ref).abs().max().item()
    assert err <= 4e-2 * max(1.0, scale), (err, scale)
    for i, t in enumerate(out):  # greedy choice fp32-consistent (within a bf16 near-tie of the oracle's max)
        row = ref[i]
        assert float(row[t]) >= float(row.max()) - 0.02 * max(1.0, float(row.abs().max())), (i, t, int(row.argmax()))
