"""Decode QKV tail folded into the decode-attention launch (attention.hip QP, ops.qkv_fold_partials): the
attention output and the newest key / value written to the paged caches must match the unfused path (split-K
partials -> RoPE / KV-write tail -> attention) and the plain-PyTorch fp32 reference (ops/reference.py), for batch
sizes on either side of the split-K shapes, contexts from one key to several pages, and short contexts where the
fold forces a second (empty) split."""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.engine.kv_cache import KVCache
from generativeaiexamples_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,Hq,Hkv,K", [(7, 32, 8, 4096), (64, 32, 8, 4096),
                                         (64, 8, 1, 8192)])  # last: a Llama-3-70B TP = 8 shard, 16 K-slices
@pytest.mark.parametrize("psw", [True, False])
def test_qkv_fold_matches_unfused_and_reference(cuda, B, Hq, Hkv, K, psw):
    torch.manual_seed(B + 100 * psw + K)
    D = 128
    N = (Hq + 2 * Hkv) * D
    max_ctx = 2600
    nbps = max_ctx // 16 + 2
    x = torch.randn(B, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    if psw:
        assert ops.preshuffle_weight(w)
    cos_sin = ops.rope_cos_sin(4096, D, 500000.0).to(cuda)
    g = torch.Generator().manual_seed(7 + B)
    ctx = torch.randint(1, max_ctx, (B,), generator=g)
    ctx[0] = 1  # a one-key context: only the new token
    if B > 2:
        ctx[1], ctx[2] = 128, 129  # one split exactly, and one key past it
    ctx = ctx.to(torch.int32).to(cuda)
    bt = torch.randperm(B * nbps, generator=g).to(torch.int32).view(B, nbps).to(cuda)
    pos = (ctx - 1).to(torch.int32)
    slots = (bt.gather(1, (pos // 16).long().view(-1, 1)).view(-1) * 16 + pos % 16).to(torch.int32)
    caches = []
    for _ in range(2):
        kv = KVCache(1, B * nbps, Hkv, D, torch.device(cuda), torch.bfloat16)
        caches.append(kv)
    caches[0].storage.normal_(generator=torch.Generator(device=cuda).manual_seed(3))
    caches[1].storage.copy_(caches[0].storage)
    ws = [ops.DecodeWorkspace(B, Hq, D, max_ctx + 64, cuda) for _ in range(2)]
    scale = 1 / math.sqrt(D)

    # unfused: split-K QKV partials -> RoPE / KV-write tail -> attention
    kc, vc = caches[0].layer(0)
    q = torch.empty(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.linear_rope_kv(x, w, None, pos, cos_sin, slots, q, kc, vc, Hq, Hkv, D)
    out_a = ops.attention_decode(q, kc, vc, bt, ctx, scale, ws=ws[0], max_ctx=max_ctx)
    # folded
    kc2, vc2 = caches[1].layer(0)
    fold = ops.qkv_fold_partials(x, w, None, kc2, D, ws[1])
    assert fold is not None, "the fold must apply to this decode shape"
    qd = torch.empty(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    out_b = ops.attention_decode(qd, kc2, vc2, bt, ctx, scale, ws=ws[1], max_ctx=max_ctx,
                                 qkv_fold=(fold[0], fold[1], pos, cos_sin, slots))
    torch.cuda.synchronize()
    # the caches agree everywhere (the new key / value written by the split that reads them) up to a bf16 ulp of
    # the rotation's rounding
    dk = (caches[0].storage.float() - caches[1].storage.float()).abs()
    assert dk.max().item() <= 2e-2 * max(1.0, caches[0].storage.float().abs().max().item()), dk.max().item()
    assert (out_a.float() - out_b.float()).abs().max().item() < 2e-2
    # fp32 reference of the whole step on the CPU
    qkv_ref = ref.linear(x.cpu().float(), w.cpu().float())
    q_ref = torch.empty(B, Hq, D)
    kc_ref = caches[0].layer(0)[0].cpu().float().clone()
    vc_ref = caches[0].layer(0)[1].cpu().float().clone()
    k_old = caches[0].layer(0)[0].cpu().float()  # already holds the new key; reference rewrites it the same way
    ref.rope_kv_write(qkv_ref, pos.cpu(), cos_sin.cpu(), slots.cpu(), q_ref, kc_ref, vc_ref, Hq, Hkv, D)
    assert (kc_ref - k_old).abs().max().item() < 5e-2
    o_ref = ref.attention_decode(q_ref, kc_ref, vc_ref, bt.cpu(), ctx.cpu(), scale)
    err = (out_b.float().cpu() - o_ref.float()).abs().max().item()
    assert err < 3e-2, err


def test_qkv_fold_in_graph_replay(cuda, monkeypatch):
    """The folded path in the engine, eager and inside captured multi-step decode graphs: every greedy token is the
    fp32 reference argmax of its prefix up to a bf16 near-tie."""
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    used = [0]
    orig = ops.qkv_fold_partials

    def spy(*a, **k):
        r = orig(*a, **k)
        used[0] += r is not None
        return r

    monkeypatch.setattr(ops, "qkv_fold_partials", spy)
    cfg = LlamaConfig.tiny(num_heads=8, num_kv_heads=2, head_dim=128, hidden_size=4096, intermediate_size=4096,
                           vocab_size=1024)
    m = LlamaModel(cfg, device="cuda").random_init(4)
    tok = small_byte_tokenizer(1024)
    # 6 sequences: decode batches > 4 take the split-K path (batch <= 4 runs the GEMV kernels)
    prompts = [list(range(3 + i, 3 + i + n)) for i, n in enumerate((5, 140, 300, 17, 129, 64))]
    sp = SamplingParams(temperature=0.0, max_tokens=24, ignore_eos=True)
    outs = {}
    for graphs in (False, True):
        eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=8, num_blocks=256, max_model_len=512, use_graphs=graphs,
                                             graph_batch_sizes=(4, 8)))
        if graphs:
            eng.capture_graphs(max_bs=8)
        outs[graphs] = [r.output_ids for r in eng.generate(prompts, sp)]
        if graphs:
            assert eng.stats["graph_steps"] > 0
    assert used[0] > 0, "the folded decode path never ran"
    for graphs, res in outs.items():  # fp32-consistent greedy tokens, eager and graph-replayed
        for p, o in zip(prompts, res):
            lg = m.reference_forward(torch.tensor(p + o[:-1]))[len(p) - 1:]
            for i, t in enumerate(o):
                row = lg[i]
                assert float(row[t]) >= float(row.max()) - 0.02 * max(1.0, float(row.abs().max())), (graphs, i, t)
