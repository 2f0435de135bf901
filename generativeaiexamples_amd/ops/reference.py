"""Plain-PyTorch fp32 reference implementations of every native op.

These define the semantics the HIP kernels are tested against (tests compare the
gfx950 kernels with these on random inputs) and they are the execution path for
CPU tensors (BASELINE config 1, the CPU plumbing config, and the CPU test tier).
Layouts are identical to the native ones:

* paged K cache  ``[num_blocks, Hkv, 16, D]``
* paged V^T cache ``[num_blocks, Hkv, D, 16]``
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

BLOCK = 16


def rms_norm(x, w, eps, residual=None):
    if residual is not None:
        r = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(r)
        x = r
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def layer_norm(x, w, b, eps, residual=None):
    if residual is not None:
        r = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(r)
        x = r
    y = F.layer_norm(x.float(), (x.shape[-1],), w.float(), None if b is None else b.float(), eps)
    return y.to(x.dtype)


def linear(x, w, bias=None, residual=None, act=None, out_dtype=None):
    """y = act(x @ w^T + bias) + residual; act in {None, 'gelu', 'relu', 'quick_gelu', 'swiglu'}.

    'swiglu' expects w interleaved per 16 rows [gate16 | up16 | ...] (see
    ``interleave_gate_up``) and returns width N/2.
    """
    y = x.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = F.gelu(y)
    elif act == "relu":
        y = F.relu(y)
    elif act == "quick_gelu":
        y = y * torch.sigmoid(1.702 * y)
    elif act == "gelu_tanh":
        y = F.gelu(y, approximate="tanh")
    elif act in ("swiglu", "geglu"):
        n = y.shape[-1]
        y4 = y.reshape(*y.shape[:-1], n // 32, 2, 16)
        g = F.silu(y4[..., 0, :]) if act == "swiglu" else F.gelu(y4[..., 0, :], approximate="tanh")
        y = (g * y4[..., 1, :]).reshape(*y.shape[:-1], n // 2)
    if residual is not None:
        y = y + residual.float()
    return y.to(out_dtype or x.dtype)


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[I, K] gate and up -> [2I, K] with rows interleaved per 16 (the fused SwiGLU GEMM layout)."""
    I, K = gate.shape
    assert I % 16 == 0
    return torch.stack([gate.reshape(I // 16, 16, K), up.reshape(I // 16, 16, K)], 1).reshape(2 * I, K)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float = 500000.0, scaling: dict | None = None,
                 device=None) -> torch.Tensor:
    """fp32 table [max_pos, D] = [cos(D/2) | sin(D/2)], neox rotate-half convention.

    ``scaling`` implements the Llama-3.1 frequency-dependent rope scaling
    ({"factor", "low_freq_factor", "high_freq_factor", "original_max_position_embeddings"}).
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:
        factor = scaling.get("factor", 8.0)
        lf, hf = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        low_wl, high_wl = old / lf, old / hf
        wl = 2 * math.pi / inv
        smooth = (old / wl - lf) / (hf - lf)
        scaled = torch.where(wl > low_wl, inv / factor, inv)
        mid = (wl <= low_wl) & (wl >= high_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], -1).float().to(device)


def _to_cache(x, cache, scale):
    """Values -> cache dtype; fp8 caches hold x / scale saturated to the e4m3fn range (like the kernel)."""
    if cache.dtype == torch.float8_e4m3fn:
        return (x.float() / scale).clamp(-448.0, 448.0).to(cache.dtype)
    return x.to(cache.dtype)


def _from_cache(x, scale):
    return x.float() * scale if x.dtype == torch.float8_e4m3fn else x.float()


def rope_kv_write(qkv, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, rope=True, k_scale=1.0,
                  v_scale=1.0):
    T = qkv.shape[0]
    x = qkv.view(T, Hq + 2 * Hkv, D).float()
    q, k, v = x[:, :Hq], x[:, Hq:Hq + Hkv], x[:, Hq + Hkv:]
    if rope:
        cs = cos_sin[positions.long()]
        c, s = cs[:, None, : D // 2], cs[:, None, D // 2:]

        def rot(t):
            t = t.to(qkv.dtype).float()  # kernel rounds inputs to bf16 first (they already are)
            a, b = t[..., : D // 2], t[..., D // 2:]
            return torch.cat([a * c - b * s, b * c + a * s], -1)

        q, k = rot(q), rot(k)
    q_out.copy_(q.to(q_out.dtype).reshape(q_out.shape))
    valid = slots >= 0
    if valid.any():
        sl = slots[valid].long()
        blk, off = sl // BLOCK, sl % BLOCK
        # the kernel rounds k (after RoPE) and v to bf16 before an fp8 conversion
        k_cache[blk, :, off, :] = _to_cache(k[valid].to(qkv.dtype), k_cache, k_scale)
        v_cache[blk, :, :, off] = _to_cache(v[valid].to(qkv.dtype), v_cache, v_scale)


def gather_kv(k_cache, v_cache, block_table, n):
    """-> K [n, Hkv, D], V [n, Hkv, D] for the first n tokens of a sequence."""
    nb = (n + BLOCK - 1) // BLOCK
    blocks = block_table[:nb].long()
    k = k_cache[blocks].permute(0, 2, 1, 3).reshape(nb * BLOCK, k_cache.shape[1], k_cache.shape[3])[:n]
    v = v_cache[blocks].permute(0, 3, 1, 2).reshape(nb * BLOCK, v_cache.shape[1], v_cache.shape[2])[:n]
    return k, v


def attention_prefill(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, scale, causal=True, return_lse=False,
                      k_scale=1.0, v_scale=1.0):
    """q [Tq, Hq, D]; per sequence b the queries are the last q_len positions of ctx_lens[b] keys.
    return_lse: also return the fp32 [Tq, Hq] natural-log softmax normalisers (-1e30 for empty rows)."""
    out = torch.empty_like(q)
    lse = torch.full(q.shape[:2], -1e30, dtype=torch.float32, device=q.device)
    Hq = q.shape[1]
    Hkv = k_cache.shape[1]
    cu = cu_q.tolist()
    for b in range(len(cu) - 1):
        s, e = cu[b], cu[b + 1]
        if e == s:
            continue
        n = int(ctx_lens[b])
        k, v = gather_kv(k_cache, v_cache, block_tables[b], n)
        k = _from_cache(k, k_scale).repeat_interleave(Hq // Hkv, dim=1)
        v = _from_cache(v, v_scale).repeat_interleave(Hq // Hkv, dim=1)
        qq = q[s:e].float()
        att = torch.einsum("qhd,khd->hqk", qq, k) * scale
        if causal:
            qpos = torch.arange(n - (e - s), n, device=q.device)
            mask = torch.arange(n, device=q.device)[None, :] > qpos[:, None]
            att = att.masked_fill(mask[None], float("-inf"))
        p = att.softmax(-1)
        out[s:e] = torch.einsum("hqk,khd->qhd", p, v).to(q.dtype)
        lse[s:e] = torch.logsumexp(att, -1).transpose(0, 1)
    return (out, lse) if return_lse else out


def attention_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, k_scale=1.0, v_scale=1.0):
    """q [B, Hq, D], one token per sequence attending to its ctx_lens[b] cached keys."""
    B = q.shape[0]
    cu = torch.arange(B + 1, dtype=torch.int32)
    return attention_prefill(q, k_cache, v_cache, block_tables, cu, ctx_lens, scale, causal=True, k_scale=k_scale,
                             v_scale=v_scale)


def attention_dense(q, k, v, cu_seqlens, scale, causal):
    """Contiguous varlen attention (encoders): q/k/v [T, H, D] (k/v may have fewer heads)."""
    out = torch.empty_like(q)
    cu = cu_seqlens.tolist()
    rep = q.shape[1] // k.shape[1]
    for b in range(len(cu) - 1):
        s, e = cu[b], cu[b + 1]
        qq, kk, vv = q[s:e].float(), k[s:e].float(), v[s:e].float()
        kk, vv = kk.repeat_interleave(rep, 1), vv.repeat_interleave(rep, 1)
        att = torch.einsum("qhd,khd->hqk", qq, kk) * scale
        if causal:
            n = e - s
            att = att.masked_fill(torch.ones(n, n, dtype=torch.bool, device=q.device).triu(1)[None], float("-inf"))
        out[s:e] = torch.einsum("hqk,khd->qhd", att.softmax(-1), vv).to(q.dtype)
    return out


def sample(logits, temperature, top_p, top_k, seeds, step, generator=None):
    """Reference sampler (distributionally equivalent to the kernel, not bit-identical)."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    for i in range(B):
        x = logits[i].float()
        T = float(temperature[i])
        if T <= 0:
            out[i] = int(torch.argmax(x))
            continue
        x = x / T
        k = int(top_k[i])
        if 0 < k < V:
            kth = torch.topk(x, k).values[-1]
            x = x.masked_fill(x < kth, float("-inf"))
        p = float(top_p[i])
        if p < 1.0:
            probs = x.softmax(-1)
            sp, si = probs.sort(descending=True)
            cum = sp.cumsum(0)
            keep = (cum - sp) < p
            thr = sp[keep].min()
            x = x.masked_fill(probs < thr, float("-inf"))
        g = torch.Generator(device="cpu")
        g.manual_seed((int(seeds[i]) * 1000003 + int(step)) & 0x7FFFFFFFFFFFFFFF)
        probs = x.softmax(-1).cpu()
        out[i] = int(torch.multinomial(probs, 1, generator=g))
    return out


def token_mask(logits, rows, mask):
    V = logits.shape[1]
    bits = (mask.long().unsqueeze(-1) >> torch.arange(32, device=mask.device)) & 1  # [R, W, 32]
    allowed = bits.reshape(mask.shape[0], -1)[:, :V].bool()
    for r, row in enumerate(rows.tolist()):
        logits[row] = torch.where(allowed[r], logits[row], torch.full_like(logits[row], float("-inf")))
    return logits


def apply_penalties(logits, tok_ids, tok_cnt, n, freq, pres, rep):
    for b in range(logits.shape[0]):
        m = int(n[b])
        ids, cnt = tok_ids[b, :m].long(), tok_cnt[b, :m].float()
        v = logits[b, ids]
        r = float(rep[b])
        if r != 1.0:
            v = torch.where(v > 0, v / r, v * r)
        v = v - float(freq[b]) * cnt - (cnt > 0).float() * float(pres[b])
        logits[b, ids] = v
    return logits


def sim_topk(Q, X, bias, n_rows, k):
    s = Q.float() @ X[:n_rows].float().t() + bias[:n_rows].float()
    k = min(k, n_rows)
    v, i = torch.topk(s, k, dim=-1)
    return v, i


def moe_route(logits, k, renorm=True):
    p = logits.float().softmax(-1)
    w, ids = torch.topk(p, k, dim=-1)
    if renorm:
        w = w / w.sum(-1, keepdim=True)
    return ids.int(), w


def moe_gemm(A, a_rows, W, offs, rows_total, swiglu):
    E, N, K = W.shape
    outw = N // 2 if swiglu else N
    C = torch.empty(rows_total, outw, dtype=A.dtype)
    o = offs.tolist()
    for e in range(E):
        s, t = o[e], o[e + 1]
        if t == s:
            continue
        rows = a_rows[s:t].long() if a_rows is not None else torch.arange(s, t)
        C[s:t] = linear(A[rows], W[e], act="swiglu" if swiglu else None)
    return C


def moe_combine(Y, pos, w, residual=None):
    y = (Y[pos.long()].float() * w.float()[..., None]).sum(1)
    if residual is not None:
        y = y + residual.float()
    return y.to(Y.dtype)


def gemv(x, W, gamma=None, eps=1e-5, epi="plain", res=None, swi=None, ks=1):
    """Small-batch decode GEMV oracle (gemv.hip): optional RMSNorm of x (rounded to bf16), fp32 product, epilogue.
    ``swi``: the input is bf16(silu(g) * u) of an fp32 [M, 2K] [gate16 | up16] interleave (x unused); ``part``: the
    fp32 row sums of ``ks`` equal K parts, [ks, M, N]."""
    if swi is not None:
        g = swi.float().view(swi.shape[0], -1, 2, 16)
        xf = (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(swi.shape[0], -1).to(torch.bfloat16).float()
    else:
        xf = x.float()
    if gamma is not None:
        xf = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()).to(torch.bfloat16).float()
    if epi == "part":
        kp = xf.shape[1] // ks
        return torch.stack([xf[:, h * kp:(h + 1) * kp] @ W.float()[:, h * kp:(h + 1) * kp].t() for h in range(ks)])
    y = xf @ W.float().t()
    if epi == "f32":
        return y
    if epi == "residual":
        res.copy_((y.to(torch.bfloat16).float() + res.float()).to(res.dtype))
        return res
    if epi == "swiglu":
        g = y.view(y.shape[0], -1, 2, 16)
        return (torch.nn.functional.silu(g[:, :, 0]) * g[:, :, 1]).reshape(y.shape[0], -1).to(torch.bfloat16)
    return y.to(torch.bfloat16)


def ep_dispatch_plan(ids, world, e_local):
    """(offs [W+1], pos [T, k], a_pairs [T*k]): the pairs stably sorted by destination rank id // e_local."""
    T, k = ids.shape
    dest = (ids.reshape(-1).long() // e_local).clamp(0, world - 1)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=world)
    offs = torch.zeros(world + 1, dtype=torch.int32, device=ids.device)
    offs[1:] = counts.cumsum(0).to(torch.int32)
    pos = torch.empty(T * k, dtype=torch.int32, device=ids.device)
    pos[order] = torch.arange(T * k, dtype=torch.int32, device=ids.device)
    return offs, pos.view(T, k), order.to(torch.int32)


def ep_pack(x, ids, offs, a_pairs, world, C, e_local):
    """Send slabs [W*C, D] + local expert ids [W*C] (padding rows: sentinel e_local, zero rows)."""
    k, D = ids.shape[1], x.shape[1]
    send = torch.zeros(world * C, D, dtype=x.dtype, device=x.device)
    eid = torch.full((world * C,), e_local, dtype=torch.int32, device=x.device)
    o, flat = offs.tolist(), ids.reshape(-1).long()
    for d in range(world):
        n = min(o[d + 1] - o[d], C)
        if n > 0:
            pairs = a_pairs[o[d]:o[d] + n].long()
            send[d * C:d * C + n] = x[pairs // k]
            eid[d * C:d * C + n] = (flat[pairs] - d * e_local).to(torch.int32)
    return send, eid


def ep_combine(back, ids, pos, offs, w, residual, e_local, C):
    T, k = ids.shape
    flat = ids.reshape(-1).long()
    dest = flat // e_local
    r = pos.reshape(-1).long() - offs.long()[dest]
    keep = r < C
    rows = back[(dest * C + r.clamp(max=C - 1))].float() * (w.reshape(-1).float() * keep.float())[:, None]
    y = rows.view(T, k, -1).sum(1)
    if residual is not None:
        y = y + residual.float()
    return y.to(back.dtype)


def embedding(ids, table, vstart=0, vend=None):
    vend = table.shape[0] + vstart if vend is None else vend
    ids = ids.long()
    ok = (ids >= vstart) & (ids < vend)
    out = table[(ids - vstart).clamp(0, table.shape[0] - 1)]
    return out * ok[:, None].to(out.dtype)


def decode_advance(toks, ids, pos, ctx, slots, bt, n_valid, block):
    n = int(n_valid.reshape(-1)[0])
    p = pos[:n].long() + 1
    ids[:n] = toks[:n].to(ids.dtype)
    pos[:n] = p.to(pos.dtype)
    ctx[:n] = (p + 1).to(ctx.dtype)
    rows = torch.arange(n, device=bt.device)
    slots[:n] = (bt[rows, p // block].long() * block + p % block).to(slots.dtype)


def pool(h, cu_seqlens, mode="mean", normalize=True):
    cu = cu_seqlens.tolist()
    outs = []
    for b in range(len(cu) - 1):
        s, e = cu[b], cu[b + 1]
        x = h[s:e].float()
        if mode == "mean":
            v = x.mean(0)
        elif mode == "cls":
            v = x[0]
        else:
            v = x[-1]
        outs.append(v)
    o = torch.stack(outs) if outs else h.new_zeros(0, h.shape[-1], dtype=torch.float32)
    if normalize:
        o = F.normalize(o, dim=-1, eps=1e-12)
    return o


def silu_mul(x):
    i = x.shape[-1] // 2
    return (F.silu(x[..., :i].float()) * x[..., i:].float()).to(x.dtype)


def gelu(x):
    return F.gelu(x.float()).to(x.dtype)


def gelu_tanh(x):
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def geglu_interleaved(x):
    n = x.shape[-1]
    x4 = x.float().reshape(*x.shape[:-1], n // 32, 2, 16)
    return (F.gelu(x4[..., 0, :], approximate="tanh") * x4[..., 1, :]).reshape(*x.shape[:-1], n // 2).to(x.dtype)


# ---------------------------------------------------------------------------------------------- fp8
FP8_MAX = 448.0


def quant_rows_fp8(x: torch.Tensor):
    """Per-row dynamic e4m3fn quantisation: (q [.., K] float8_e4m3fn, scale [rows] fp32 = amax/448)."""
    xf = x.float().reshape(-1, x.shape[-1])
    s = xf.abs().amax(-1).clamp_min(1e-12) / FP8_MAX
    # x * (1 / s) in fp32, as the kernel (a reciprocal multiply, not a division per element)
    q = (xf * (1.0 / s)[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q.reshape(x.shape), s


def linear_fp8(xq, sx, wq, sw, bias=None, residual=None, act=None, out_dtype=torch.bfloat16):
    """fp32 reference of the fp8 GEMM: dequantise both operands, then ``linear``."""
    x = xq.float().reshape(-1, xq.shape[-1]) * sx.reshape(-1, 1)
    w = wq.float() * sw.reshape(-1, 1)
    y = linear(x, w, bias, None if residual is None else residual.reshape(x.shape[0], -1), act, torch.float32)
    return y.reshape(*xq.shape[:-1], y.shape[-1]).to(out_dtype)


# ---------------------------------------------------------------------------------------------- vision
def patchify(img: torch.Tensor, P: int, mean: torch.Tensor, inv_std: torch.Tensor, Kp: int) -> torch.Tensor:
    """[B, C, H, W] fp32 -> normalised patches [B * gh * gw, Kp] bf16, (c, ky, kx) order, zero padded."""
    B, C, H, W = img.shape
    x = (img.float() - mean[:C].view(1, C, 1, 1)) * inv_std[:C].view(1, C, 1, 1)
    x = x.reshape(B, C, H // P, P, W // P, P).permute(0, 2, 4, 1, 3, 5).reshape(B * (H // P) * (W // P), C * P * P)
    out = torch.zeros(x.shape[0], Kp, dtype=torch.bfloat16)
    out[:, : C * P * P] = x.to(torch.bfloat16)
    return out


def vit_embed(patches: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor, B: int) -> torch.Tensor:
    D = cls.numel()
    p = patches.float().reshape(B, -1, D)
    x = torch.cat([cls.float().view(1, 1, D).expand(B, 1, D), p], 1) + pos.float()[: p.shape[1] + 1]
    return x.reshape(-1, D).to(torch.bfloat16)
