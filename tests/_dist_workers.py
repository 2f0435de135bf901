"""Worker bodies for the multi-process (gloo, 127.0.0.1) distributed tests."""
import os

import torch
import torch.distributed as dist


# A one-GPU multi-rank rehearsal's ranks spin-wait on each other inside peer-memory collectives, so every rank's
# kernel must be resident on the GPU at the same time. The hardware scheduler maps a bounded number of hardware
# queues at once: 8 processes x HIP's default 4 queues oversubscribe it and the ranks are time-sliced (profiles/r4/
# custom_ar_a2a.log: 23 ms per 1 MiB all-reduce at world 8 vs 83 us at world 4). One queue per process keeps 8 ranks
# mapped; the long spin bound covers ranks that reach a collective seconds apart on a few shared CPU cores.
CORESIDENT_US = 2000.0  # a probe all-reduce slower than this per call means the ranks are time-sliced


def one_gpu_rank_env(world: int = 8):
    """Set before the process's first HIP call (spawned workers: at the top of the worker body). The all-to-all's
    looping grid is capped so that every rank's spin-waiting workgroups fit on the one GPU together (2048 resident
    256-thread workgroups on 256 CUs, csrc/comm/custom_ar.hip ar_max_grid)."""
    os.environ["GPU_MAX_HW_QUEUES"] = "1"
    os.environ["GAI_AR_SPIN_LOG2"] = "29"
    os.environ["GAI_AR_MAX_GRID"] = str(max(1, min(512, 2048 // max(1, world))))


def coresidency_probe(car, dev, out_dir, tag, rank, iters=20):
    """Co-residency as a checked precondition: us per 64 KiB peer-memory all-reduce, every rank launching together.
    Co-resident ranks finish one in tens of us; time-sliced ranks need a scheduler quantum (ms) per call. Writes
    <tag>_probe_<rank>.json (the test compares it against CORESIDENT_US and prints the KFD census when it fails)."""
    import json
    import time as _time

    x = torch.zeros(32768, dtype=torch.bfloat16, device=dev)
    car.all_reduce(x)
    torch.cuda.synchronize()
    dist.barrier(group=car.group)
    t0 = _time.perf_counter()
    for _ in range(iters):
        car.all_reduce(x)
    torch.cuda.synchronize()
    us = (_time.perf_counter() - t0) * 1e6 / iters
    car.check()
    with open(os.path.join(out_dir, f"{tag}_probe_{rank}.json"), "w") as f:
        json.dump({"us_per_call": us, "pid": os.getpid(), "queues_env": os.environ.get("GPU_MAX_HW_QUEUES")}, f)
    return us


def _init(rank, world, port, tp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from generativeaiexamples_amd.parallel import dist as gdist

    return gdist.init_distributed(tp_size=tp, backend="gloo")


def tp_llama_worker(rank, world, port, out_dir, overlap_rows=None):
    if overlap_rows:  # exercise the row-chunked overlapped all-reduce path on these short prompts
        os.environ["GAI_TP_OVERLAP_CHUNK_ROWS"] = str(overlap_rows)
    ctx = _init(rank, world, port, world)
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext

    cfg = LlamaConfig.tiny(num_heads=4, num_kv_heads=2, vocab_size=512)
    ref = LlamaModel(cfg, device="cpu", dist_ctx=DistContext()).random_init(5)  # same on every rank
    sd = ref.export_hf_state()
    m = LlamaModel(cfg, device="cpu", dist_ctx=ctx).load_hf_state(sd)
    tok = small_byte_tokenizer(512)
    prompts = [list(range(7, 7 + n)) for n in (11, 40)]
    outs = []
    for model in (m, ref):
        eng = LLMEngine(model, tok, EngineConfig(num_blocks=64, max_model_len=256, use_graphs=False))
        for p in prompts:
            eng.add_request(p, SamplingParams(temperature=0.0, max_tokens=1))
        b = eng.sched.schedule()
        fb, _ = eng._make_batch(b)
        outs.append(model.forward(fb, eng.kv).float())
    torch.save({"tp": outs[0], "ref": outs[1]}, os.path.join(out_dir, f"tp_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def ep_worker(rank, world, port, out_dir):
    _init(rank, world, port, 1)
    from generativeaiexamples_amd import ops
    from generativeaiexamples_amd.parallel import ep

    E, D, I, k = 4, 64, 32, 2
    g = torch.Generator().manual_seed(3)
    w13 = (torch.randn(E, 2 * I, D, generator=g) / 8).to(torch.bfloat16)
    w2 = (torch.randn(E, D, I, generator=g) / 6).to(torch.bfloat16)
    x_all = torch.randn(2, 9, D, generator=g).to(torch.bfloat16)
    logit_all = torch.randn(2, 9, E, generator=g)
    x, logits = x_all[rank], logit_all[rank]
    ids, w = ops.moe_route(logits, k)
    e_local = E // world
    # the prefill-sized step's exchange: capacity T * k (nothing dropped), per-peer counts on the device
    rows, eid, plan = ep.dispatch_padded(x, ids, E, None, None, exact_counts=True)
    y = ep.local_experts_padded(rows, eid, w13[rank * e_local:(rank + 1) * e_local],
                                w2[rank * e_local:(rank + 1) * e_local])
    out = ep.combine_padded(y, w, plan, None)
    # single-process oracle with all experts
    a_rows, offs, pos = ops.moe_dispatch(ids, E)
    h1 = ops.moe_gemm(x, a_rows, w13, offs, x.shape[0] * k, True)
    yy = ops.moe_gemm(h1, None, w2, offs, x.shape[0] * k, False)
    exp = ops.moe_combine(yy, pos, w)
    torch.save({"out": out.float(), "exp": exp.float()}, os.path.join(out_dir, f"ep_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def ep_padded_worker(rank, world, port, out_dir):
    """Sync-free fixed-capacity EP exchange (graph-capturable decode path) vs the single-process oracle."""
    _init(rank, world, port, 1)
    from generativeaiexamples_amd import ops
    from generativeaiexamples_amd.parallel import ep

    E, D, I, k = 8, 64, 32, 2
    g = torch.Generator().manual_seed(5)
    w13 = (torch.randn(E, 2 * I, D, generator=g) / 8).to(torch.bfloat16)
    w2 = (torch.randn(E, D, I, generator=g) / 6).to(torch.bfloat16)
    x_all = torch.randn(world, 7, D, generator=g).to(torch.bfloat16)
    logit_all = torch.randn(world, 7, E, generator=g)
    x, logits = x_all[rank], logit_all[rank]
    ids, w = ops.moe_route(logits, k)
    e_local = E // world
    mine = slice(rank * e_local, (rank + 1) * e_local)
    rows, eid, plan = ep.dispatch_padded(x, ids, E, None, None)
    assert rows.shape[0] == world * 7 * k
    # device-side count exchange: rank r sends (r + 2 q) % 5 to rank q, so it receives (q + 2 r) % 5 from q
    got = ep.exchange_counts(torch.tensor([(rank + 2 * q) % 5 for q in range(world)], dtype=torch.int32), None)
    assert got.tolist() == [(q + 2 * rank) % 5 for q in range(world)], got
    y = ep.local_experts_padded(rows, eid, w13[mine], w2[mine])
    out = ep.combine_padded(y, w, plan, None)
    a_rows, offs, pos = ops.moe_dispatch(ids, E)
    h1 = ops.moe_gemm(x, a_rows, w13, offs, x.shape[0] * k, True)
    exp = ops.moe_combine(ops.moe_gemm(h1, None, w2, offs, x.shape[0] * k, False), pos, w)
    # a capacity of 1 row per peer drops pairs: their contribution is zero, never garbage
    rows1, eid1, plan1 = ep.dispatch_padded(x, ids, E, 1, None)
    out1 = ep.combine_padded(ep.local_experts_padded(rows1, eid1, w13[mine], w2[mine]), w, plan1, None)
    torch.save({"out": out.float(), "exp": exp.float(), "out1": out1.float()},
               os.path.join(out_dir, f"ep_padded_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def sharded_index_worker(rank, world, port, out_dir, max_queries=None):
    _init(rank, world, port, 1)
    from generativeaiexamples_amd.index.hbm_index import HBMIndex
    from generativeaiexamples_amd.index.sharded import ShardedIndex

    g = torch.Generator().manual_seed(0)
    full = torch.nn.functional.normalize(torch.randn(2 * 300, 32, generator=g), dim=-1)
    queries = torch.nn.functional.normalize(torch.randn(2 * 5, 32, generator=g), dim=-1)
    shard = full[rank * 300:(rank + 1) * 300]
    idx = HBMIndex(32, "cosine", device="cpu", capacity=16)
    idx.add(shard)
    si = ShardedIndex(idx, max_queries=max_queries)
    my_q = queries[rank * 5:(rank + 1) * 5]
    if max_queries is not None:  # uneven per-rank batches under the padded (sync-free) protocol
        my_q = my_q[: 5 - rank]
    rel, rows = si.search_raw(my_q, 4)
    bf = lambda t: t.to(torch.bfloat16).float()  # noqa: E731  (the index stores bf16 vectors)
    exp = torch.topk(bf(my_q) @ bf(full).t(), 4, dim=-1)
    got_global = [[ShardedIndex.split_row(int(x))[0] * 300 + ShardedIndex.split_row(int(x))[1] for x in r]
                  for r in rows.tolist()]
    torch.save({"got": got_global, "exp": exp.indices.tolist(), "rel": rel, "exp_v": exp.values},
               os.path.join(out_dir, f"idx_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def fault_worker(rank, world, port, out_dir, mode):
    """mode 'kill': rank 1 dies at its 3rd collective; rank 0 must get RankFailure (not hang).
    mode 'delay': rank 1 sleeps 300 ms before every collective; rank 0 observes the delay."""
    import time

    if mode == "kill":
        os.environ.update(FI_KILL_RANK="1", FI_KILL_AT_CALL="3", GAI_DIST_TIMEOUT_S="30")
    else:
        os.environ.update(FI_DELAY_ALLREDUCE_MS="300", FI_DELAY_RANK="1")
    from generativeaiexamples_amd.parallel import fault

    fault.INJECTOR.reload()
    ctx = _init(rank, world, port, 2)
    t = torch.ones(8)
    status, t0 = "ok", time.perf_counter()
    try:
        for _ in range(6):
            ctx.tp_all_reduce(t)
    except fault.RankFailure as e:
        status = "rank_failure: " + str(e)[:200]
    dt = time.perf_counter() - t0
    with open(os.path.join(out_dir, f"fault_{mode}_{rank}.txt"), "w") as f:
        f.write(f"{status}\n{dt}\n{t[0].item()}\n")
    if mode == "delay":
        dist.destroy_process_group()
    else:
        os._exit(0)  # the peer is gone: skip teardown of the broken group


def lora_tp_worker(rank, world, port, out_dir):
    """TP=2 differentiable forward + LoRA grads vs the single-process values of the same weights."""
    ctx = _init(rank, world, port, 2)
    from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext
    from generativeaiexamples_amd.training.forward import lm_loss
    from generativeaiexamples_amd.training.lora import LoRAAdapter, LoRAConfig

    torch.manual_seed(0)
    cfg = LlamaConfig.tiny(num_layers=2)
    full = LlamaModel(cfg, device="cpu", dist_ctx=DistContext()).random_init(seed=3)
    for t in full.w.values():
        t.data = t.data.float()
    sd = full.export_hf_state()
    tp = LlamaModel(cfg, device="cpu", dist_ctx=ctx, dtype=torch.float32).load_hf_state(sd)
    lcfg = LoRAConfig(r=4, alpha=8, targets=("qkv", "o", "gate_up", "down"))
    ad_full = LoRAAdapter(full, lcfg, seed=1)
    ad_tp = LoRAAdapter(tp, lcfg, seed=1)
    with torch.no_grad():  # non-zero B so the LoRA path matters; shard full adapters the way weights are
        for j, (k, v) in enumerate(ad_full.params.items()):
            if k.endswith(".B"):  # deterministic across processes (str hash is randomised per process)
                v.normal_(0, 0.05, generator=torch.Generator().manual_seed(j))
        for k, v in ad_tp.params.items():
            src = ad_full.params[k]
            t = k.split(".")[1]
            if src.shape == v.shape:
                v.copy_(src)
            elif t in ("qkv", "gate_up"):  # column-parallel: B rows sharded like the weight rows
                if t == "qkv":
                    hd, H, Hkv = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
                    q, kk, vv = src.split([H * hd, Hkv * hd, Hkv * hd])
                    parts = [x.chunk(world)[rank] for x in (q, kk, vv)]
                    v.copy_(torch.cat(parts))
                else:
                    v.copy_(src.view(world, -1, src.shape[1])[rank])
            else:  # row-parallel A: columns sharded
                v.copy_(src.view(src.shape[0], world, -1)[:, rank])
    ids = torch.randint(3, cfg.vocab_size, (2, 24), generator=torch.Generator().manual_seed(5))
    labels = ids.clone()
    labels[:, :8] = -100
    l_full = lm_loss(full, ad_full, ids, labels)
    l_full.backward()
    l_tp = lm_loss(tp, ad_tp, ids, labels)
    l_tp.backward()
    for p in ad_tp.tp_replicated():
        dist.all_reduce(p.grad, group=ctx.tp_group)
    # compare the gradient of one replicated and one sharded factor
    g_rep = ad_tp.params["l1.o.B"].grad
    g_rep_ref = ad_full.params["l1.o.B"].grad
    torch.save({"loss": l_tp.detach(), "loss_ref": l_full.detach(), "g": g_rep, "g_ref": g_rep_ref,
                "gA": ad_tp.params["l0.qkv.A"].grad, "gA_ref": ad_full.params["l0.qkv.A"].grad},
               os.path.join(out_dir, f"lora_tp_{rank}.pt"))
    dist.barrier()
    os._exit(0)  # skip gloo teardown (sporadic abort after autograd-issued collectives); results are saved


def lora_dp_worker(rank, world, port, out_dir):
    """DP=2 LoRA SFT with the overlapped gradient bucketer: replicas stay identical, loss falls."""
    ctx = _init(rank, world, port, 1)
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.training.lora import LoRAConfig
    from generativeaiexamples_amd.training.trainer import LoRATrainer, TrainConfig

    cfg = LlamaConfig.tiny(num_layers=2)
    m = LlamaModel(cfg, device="cpu", dist_ctx=ctx, dtype=torch.float32).random_init(seed=3)
    tr = LoRATrainer(m, small_byte_tokenizer(cfg.vocab_size), LoRAConfig(r=4, alpha=8),
                     TrainConfig(steps=12, global_batch=4, micro_batch=1, seq_len=64, lr=3e-3, warmup=2))
    hist = tr.train()
    torch.save({"hist": torch.tensor(hist), "A": tr.lora.params["l0.qkv.A"].detach().clone(),
                "launched": tr.bucketer.launched}, os.path.join(out_dir, f"lora_dp_{rank}.pt"))
    dist.barrier()
    os._exit(0)


def embed_ft_dp_worker(rank, world, port, out_dir):
    """DP=2 contrastive fine-tuning of a tiny encoder (gloo): replicas stay identical, loss falls."""
    _init(rank, world, port, 1)
    torch.manual_seed(0)
    from generativeaiexamples_amd.engine.embedder import Embedder
    from generativeaiexamples_amd.engine.tokenizer import bert_byte_tokenizer
    from generativeaiexamples_amd.models.bert import BertConfig, BertModel
    from generativeaiexamples_amd.training.embed_ft import EmbedFineTuner, EmbedFTConfig, synthetic_pairs

    enc = BertModel(BertConfig.tiny(num_layers=1), device="cpu").random_init(rank)  # rank 0's weights broadcast
    emb = Embedder(enc, bert_byte_tokenizer(2048))
    cfg = EmbedFTConfig(global_batch=16, micro_batch=4, lr=2e-4, max_steps=6, gather_negatives=True, tau=0.05)
    ft = EmbedFineTuner(emb, cfg, synthetic_pairs(64))
    hist = ft.fit()
    torch.save({"hist": torch.tensor(hist), "w": ft.w["l0.qkv"].detach().clone()},
               os.path.join(out_dir, f"eft_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def tp_sp_worker(rank, world, port, out_dir):
    """TP=2 with sequence parallelism (reduce-scatter / all-gather) == TP=2 all-reduce == TP=1, on a mixed
    prefill + decode batch whose token count is not a multiple of tp."""
    ctx = _init(rank, world, port, world)
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext

    outs = {}
    for name, kw in (("llama", {}), ("starcoder2", dict(arch="starcoder2", norm="layernorm", mlp="gelu_tanh",
                                                        qkv_bias=True, o_bias=True, mlp_bias=True))):
        cfg = LlamaConfig.tiny(num_heads=4, num_kv_heads=2, vocab_size=512, **kw)
        ref = LlamaModel(cfg, device="cpu", dist_ctx=DistContext()).random_init(9)
        sd = ref.export_hf_state()
        m = LlamaModel(cfg, device="cpu", dist_ctx=ctx).load_hf_state(sd)
        tok = small_byte_tokenizer(512)
        res = {}
        for mode in ("ref", "tp", "sp"):
            model = ref if mode == "ref" else m
            ctx.sequence_parallel = mode == "sp"
            eng = LLMEngine(model, tok, EngineConfig(num_blocks=64, max_model_len=256, use_graphs=False,
                                                     decode_steps=1))
            first = eng.add_request(list(range(5, 16)), SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True))
            if eng.leader:  # TP engine: rank 0 plans the step, the follower executes the same plan
                eng.step()  # prefill of the first request
                eng.release_followers()
            else:
                assert eng.follow() == "yield"
            eng.add_request(list(range(7, 7 + 26)), SamplingParams(temperature=0.0, max_tokens=1))
            if eng.leader:  # only the leader's scheduler is authoritative: ship its plan to the follower
                plan = eng._plan_eager(eng.sched.schedule())  # 1 decode token + 26 prefill tokens = 27 (odd)
                if eng.chan is not None:
                    eng.chan.send(plan)
            else:
                plan = eng.chan.recv()
            assert len(plan["arr"][0]) == 27
            fb = eng._batch_from_plan(plan)
            res[mode] = model.forward(fb, eng.kv).float()
            del first
        ctx.sequence_parallel = False
        outs[name] = res
    torch.save(outs, os.path.join(out_dir, f"sp_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def custom_ar_worker(rank, world, port, out_dir):
    """Every rank on cuda:0 (one-GPU box), gloo for the handle exchange: the one-shot peer-memory
    all-reduce must equal the fp32 sum of every rank's input, eagerly (bf16 + fp32, in/out of
    place, sizes across chunk boundaries, repeated calls over both parities) and from a captured
    HIP graph replayed with new inputs. Writes one status line per rank."""
    import json

    one_gpu_rank_env(world)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from generativeaiexamples_amd.parallel.custom_ar import CustomAllReduce

    car = CustomAllReduce(None, dev, max_bytes=4 << 20, a2a_max_bytes=12 << 20)
    coresidency_probe(car, dev, out_dir, "car", rank)
    errs = []

    def inputs(n, dtype, seed):
        g = torch.Generator().manual_seed(seed)
        xs = [torch.randn(n, generator=g).to(dtype) for _ in range(world)]
        ref = torch.stack([x.float() for x in xs]).sum(0)
        return xs[rank].to(dev), ref

    sizes = [8, 64, 2048, 8192, 8200, 65536 + 8, 524288, (4 << 20) // 2]  # elements (bf16)
    for it, n in enumerate(sizes * 2):  # twice: both buffer parities per block
        for dtype in (torch.bfloat16, torch.float32):
            if n * (2 if dtype == torch.bfloat16 else 4) > car.max_bytes:
                continue
            x, ref = inputs(n, dtype, 100 * it + (dtype == torch.float32))
            torch.cuda.synchronize()
            dist.barrier()  # ranks time-slice ONE GPU here: launch together so no spin outlives its peer's host
            if it % 2:
                y = car.all_reduce(x)  # in place
            else:
                y = torch.empty_like(x)
                car.all_reduce(x, y)
            torch.cuda.synchronize()
            tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
            e = (y.float().cpu() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
            if not e < tol:
                errs.append(f"n={n} {dtype} rel err {e}")
    # explicit algorithms: two-shot (reduce-scatter + all-gather) and one-shot on the same messages
    for it, n in enumerate([world * 8, world * 4096, world * 8192 + world * 8, 1 << 20, (4 << 20) // 4]):
        for algo in ("twoshot", "oneshot"):
            for dtype in (torch.bfloat16, torch.float32):
                nbytes = n * (2 if dtype == torch.bfloat16 else 4)
                if nbytes > car.max_bytes or nbytes % (16 * world):
                    continue
                x, ref = inputs(n, dtype, 500 + 10 * it + (dtype == torch.float32))
                torch.cuda.synchronize()
                dist.barrier()
                y = car.all_reduce(x.clone(), algo=algo)
                torch.cuda.synchronize()
                tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
                e = (y.float().cpu() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                if not e < tol:
                    errs.append(f"{algo} n={n} {dtype} rel err {e}")
    # fused all-reduce + residual add + RMSNorm vs the unfused rounding
    for D in (2048, 4096, 8192):
        for T in (1, 7, 64):
            g0 = torch.Generator().manual_seed(D + T)
            xs = [torch.randn(T, D, generator=g0).to(torch.bfloat16) for _ in range(world)]
            res0 = torch.randn(T, D, generator=g0).to(torch.bfloat16)
            wn = (torch.rand(D, generator=g0) + 0.5).to(torch.bfloat16)
            h = torch.stack([x.float() for x in xs]).sum(0).to(torch.bfloat16)
            r = (h.float() + res0.float()).to(torch.bfloat16)
            want = (r.float() * torch.rsqrt(r.float().pow(2).mean(-1, keepdim=True) + 1e-5) * wn.float())
            res = res0.to(dev)
            torch.cuda.synchronize()
            dist.barrier()
            y = car.all_reduce_rmsnorm(xs[rank].to(dev), res, wn.to(dev), 1e-5)
            torch.cuda.synchronize()
            if not torch.equal(res.cpu(), r):
                errs.append(f"ar_rmsnorm D={D} T={T}: residual differs from bf16(h + res)")
            e = (y.float().cpu() - want).abs().max().item()
            if not e < 3e-2 * want.abs().max().item():
                errs.append(f"ar_rmsnorm D={D} T={T} err {e}")
    # one-shot all-to-all (expert-parallel token exchange) on the same buffers, interleaved with all-reduces:
    # segment q of rank r carries (r, q) tags; the result's segment q must be rank q's segment `rank`
    for seg in (8, 4104, 128 * 4104, (4 << 20) // 2):  # bf16 elements per peer (4104 = Mixtral row + id tail)
        if seg * 2 > car.max_bytes:
            continue
        x = torch.empty(world, seg, dtype=torch.bfloat16)
        for q in range(world):
            x[q] = float(rank * 16 + q) + torch.arange(seg, dtype=torch.float32) % 64 / 64
        torch.cuda.synchronize()
        dist.barrier()
        y = car.all_to_all(x.to(dev))
        car.all_reduce(torch.ones(1024, dtype=torch.float32, device=dev))
        torch.cuda.synchronize()
        y = y.cpu()
        for q in range(world):
            want = (float(q * 16 + rank) + torch.arange(seg, dtype=torch.float32) % 64 / 64).to(torch.bfloat16)
            if not torch.equal(y[q], want):
                errs.append(f"all_to_all seg={seg}: segment {q} wrong")
    # all-to-all of valid rows only (the expert-parallel prefill exchange): rank r sends n(r, q) of R rows to q; the
    # receiver writes only the first n(q, r) rows of segment q, the rest keep their previous contents. 1400 rows of
    # 8208 B = 11.5 MB per segment: more chunks than blocks (the blocks loop over chunks)
    for R, ncount in ((64, lambda a, b: (3 * a + 5 * b) % 65), (1400, lambda a, b: 1400 - 97 * ((a + b) % 4))):
        x = torch.empty(world, R, 4104, dtype=torch.bfloat16)
        for q in range(world):
            x[q] = (float(rank * 16 + q) + torch.arange(R, dtype=torch.float32)[:, None] / 256).to(torch.bfloat16)
        send_n = torch.tensor([ncount(rank, q) for q in range(world)], dtype=torch.int32, device=dev)
        recv_n = torch.tensor([ncount(q, rank) for q in range(world)], dtype=torch.int32, device=dev)
        out = torch.full((world, R, 4104), -7.0, dtype=torch.bfloat16, device=dev)
        torch.cuda.synchronize()
        dist.barrier()
        car.all_to_all(x.view(world * R, 4104).to(dev), out=out.view(world * R, 4104), send_rows=send_n,
                       recv_rows=recv_n)  # rows = dim-0 rows of the 2-D slab
        car.all_reduce(torch.ones(1024, dtype=torch.float32, device=dev))
        torch.cuda.synchronize()
        o = out.cpu()
        for q in range(world):
            n = ncount(q, rank)
            want = (float(q * 16 + rank) + torch.arange(n, dtype=torch.float32)[:, None] / 256).to(torch.bfloat16)
            if not torch.equal(o[q, :n], want.expand(n, 4104)):
                errs.append(f"all_to_all rows R={R}: segment {q} valid rows wrong")
            if not torch.all(o[q, n:] == -7.0).item():
                errs.append(f"all_to_all rows R={R}: segment {q} rows past the count were written")
    # graph capture: three chained all-reduces on static buffers, replayed with new inputs
    n = 64 * 4096
    static = torch.zeros(n, dtype=torch.bfloat16, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        car.all_reduce(static)  # warm (also advances the epoch counters identically on every rank)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    big = torch.zeros(1 << 20, dtype=torch.bfloat16, device=dev)
    with torch.cuda.stream(s):
        car.all_reduce(big, algo="twoshot")  # warm the two-shot epochs too
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        car.all_reduce(static)
        static.mul_(0.5)
        car.all_reduce(static)
        car.all_reduce(big, algo="twoshot")
    for rep in range(4):
        x, ref = inputs(n, torch.bfloat16, 7000 + rep)
        static.copy_(x)
        torch.cuda.synchronize()
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        want = ref * 0.5 * world
        e = (static.float().cpu() - want).abs().max().item() / (want.abs().max().item() + 1e-6)
        if not e < 3e-2:
            errs.append(f"graph replay {rep} rel err {e}")
        if rep == 0:
            big.fill_(1.0)
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            if not torch.all(big.float().cpu() == float(world)).item():  # every rank contributed ones
                errs.append("graph replay two-shot: wrong sum")
    car.check()
    # rough latency (on a shared single GPU: all ranks time-slice one device)
    t = torch.zeros(64 * 8192, dtype=torch.bfloat16, device=dev)
    for _ in range(5):
        car.all_reduce(t)
    torch.cuda.synchronize()
    dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(50):
        car.all_reduce(t)
    ev1.record()
    torch.cuda.synchronize()
    us = ev0.elapsed_time(ev1) * 1000 / 50
    car.check()
    dist.barrier()
    car.close()
    with open(os.path.join(out_dir, f"car_{rank}.json"), "w") as f:
        json.dump({"errors": errs, "us_1MiB": us}, f)
    dist.destroy_process_group()


def cp_ring_worker(rank, world, port, out_dir, causal, device="cpu"):
    """Ring attention over `world` gloo ranks: each rank's zigzag output must match the same rows of
    full (unsharded) attention. device='cuda': every rank on cuda:0, pairs on the HIP kernel."""
    import json
    import math

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from generativeaiexamples_amd.ops import reference as ref
    from generativeaiexamples_amd.parallel import context_parallel as cp

    S, Hq, Hkv, D = 2 * world * 24, 4, 2, 64
    g = torch.Generator().manual_seed(5)
    q = torch.randn(S, Hq, D, generator=g).to(torch.bfloat16)
    k = torch.randn(S, Hkv, D, generator=g).to(torch.bfloat16)
    v = torch.randn(S, Hkv, D, generator=g).to(torch.bfloat16)
    scale = 1 / math.sqrt(D)
    cu = torch.tensor([0, S], dtype=torch.int32)
    full = ref.attention_dense(q, k, v, cu, scale, bool(causal)).float()
    dev = torch.device(device if device == "cpu" else "cuda:0")
    if dev.type == "cuda":
        torch.cuda.set_device(0)
    mine = cp.ring_attention(*(cp.zigzag_shard(t, rank, world).to(dev) for t in (q, k, v)), scale=scale,
                             causal=bool(causal)).float().cpu()
    want = cp.zigzag_shard(full, rank, world)
    err = (mine - want).abs().max().item()
    with open(os.path.join(out_dir, f"cp_{rank}.json"), "w") as f:
        json.dump({"err": err}, f)
    dist.destroy_process_group()


def tp_engine_worker(rank, world, port, out_dir):
    """TP=world serving engine (rank 0 schedules and publishes step plans, the others follow them) must
    generate exactly what a single-process engine generates: greedy and seeded sampling, chunked prefill,
    multi-step decode runs, and an abort issued on rank 0 mid-generation. fp32 weights so the TP partial
    sums cannot flip a near-tie."""
    import json

    ctx = _init(rank, world, port, world)
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext

    cfg = LlamaConfig.tiny(num_heads=8, num_kv_heads=8, head_dim=32, hidden_size=256, intermediate_size=512,
                           vocab_size=512)
    ref = LlamaModel(cfg, device="cpu", dtype=torch.float32, dist_ctx=DistContext()).random_init(11)
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32, dist_ctx=ctx).load_hf_state(ref.export_hf_state())
    tok = small_byte_tokenizer(512)
    ecfg = dict(num_blocks=96, max_model_len=256, use_graphs=False, decode_steps=4, max_num_seqs=8,
                max_batched_tokens=48, prefill_chunk=32, prefix_cache=False)
    eng = LLMEngine(m, tok, EngineConfig(**ecfg))
    if not eng.leader:
        assert eng.follow() == "stop"
        dist.barrier()
        dist.destroy_process_group()
        return
    prompts = [list(range(9 + i, 9 + i + n)) for i, n in enumerate((5, 37, 61, 18))]
    sps = [SamplingParams(temperature=0.0, max_tokens=n, ignore_eos=True) for n in (9, 14, 6, 11)]
    sps[3] = SamplingParams(temperature=0.8, top_p=0.9, max_tokens=11, ignore_eos=True, seed=1234)

    def drive(e):  # same request stream and the same abort point on both engines (same seeds / step counts)
        reqs = [e.add_request(p, sp, request_id=f"r{i}") for i, (p, sp) in enumerate(zip(prompts, sps))]
        victim = e.add_request(list(range(100, 150)), SamplingParams(temperature=0.0, max_tokens=40,
                                                                     ignore_eos=True), request_id="victim")
        steps = 0
        while e.has_work():
            e.step()
            steps += 1
            if steps == 4:
                assert e.abort("victim")
        return reqs, victim

    reqs, victim = drive(eng)
    free_ok = eng.sched.num_free_blocks() == eng.sched.num_blocks()
    multi = eng.stats["multi_step_runs"]
    eng.release_followers(stop=True)
    single, _ = drive(LLMEngine(ref, tok, EngineConfig(**ecfg)))
    with open(os.path.join(out_dir, "tp_engine.json"), "w") as f:
        json.dump({"tp": [r.output_ids for r in reqs], "ref": [r.output_ids for r in single],
                   "victim": victim.finish_reason, "victim_len": len(victim.output_ids), "free_ok": free_ok,
                   "multi": multi, "plans": eng.chan.sent}, f)
    dist.barrier()
    dist.destroy_process_group()


def write_tiny_llama_ckpt(path, seed=21):
    """A tiny Llama in HF layout (config.json + model.safetensors) for checkpoint-serving tests."""
    import json

    from safetensors.torch import save_file

    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext

    cfg = LlamaConfig.tiny(num_heads=8, num_kv_heads=4, head_dim=32, hidden_size=256, intermediate_size=512,
                           vocab_size=512)
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32, dist_ctx=DistContext()).random_init(seed)
    os.makedirs(path, exist_ok=True)
    save_file({k: v.contiguous() for k, v in m.export_hf_state().items()}, os.path.join(path, "model.safetensors"))
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump({"model_type": "llama", "vocab_size": 512, "hidden_size": 256, "intermediate_size": 512,
                   "num_hidden_layers": cfg.num_layers, "num_attention_heads": 8, "num_key_value_heads": 4,
                   "head_dim": 32, "max_position_embeddings": 2048, "rms_norm_eps": cfg.rms_eps,
                   "rope_theta": cfg.rope_theta, "bos_token_id": 1, "eos_token_id": 2,
                   "tie_word_embeddings": False}, f)


def tp_serving_worker(rank, world, port, out_dir, ckpt):
    """`/v1` serving of a TP=world generator: rank 0 runs the API (ServiceHub + FastAPI), the other ranks
    follow its step plans; completions must equal a single-process engine on the same checkpoint, a
    client-side abort mid-stream must not desynchronise the ranks, and shutdown must end the followers."""
    import json

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from generativeaiexamples_amd.serving.hub import HubSpec, ServiceHub

    spec = HubSpec(llm="tiny-llama", llm_weights=ckpt, embedder=None, device="cpu", tp=world, dtype="float32",
                   max_num_seqs=8, max_model_len=512, max_batched_tokens=64, use_graphs=False)
    hub = ServiceHub.build(spec)
    if hub.is_follower:
        assert hub.serve_follower() == "stop"
        dist.barrier()
        dist.destroy_process_group()
        return
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import apply_chat_template
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext
    from generativeaiexamples_amd.serving.openai_api import create_openai_app

    msgs = [[{"role": "user", "content": f"question {i}: " + "x" * (7 * i)}] for i in range(3)]
    res = {"api": [], "stream_ok": False}
    with TestClient(create_openai_app(hub)) as c:
        for m in msgs:
            r = c.post("/v1/chat/completions", json={"messages": m, "max_tokens": 12, "temperature": 0,
                                                      "ignore_eos": True})
            assert r.status_code == 200, r.text
            res["api"].append(r.json()["choices"][0]["message"]["content"])
        # client disconnects after two chunks: the request is aborted on rank 0 only
        with c.stream("POST", "/v1/chat/completions", json={"messages": msgs[0], "max_tokens": 200, "stream": True,
                                                             "ignore_eos": True}) as s:
            for i, _ in enumerate(s.iter_lines()):
                if i > 2:
                    break
        r = c.post("/v1/chat/completions", json={"messages": msgs[1], "max_tokens": 12, "temperature": 0,
                                                  "ignore_eos": True})
        res["after_abort"] = r.json()["choices"][0]["message"]["content"]
    tok = hub.llm().tokenizer
    hub.shutdown()
    ref = LlamaModel(LlamaConfig.from_hf(ckpt), device="cpu", dtype=torch.float32,
                     dist_ctx=DistContext()).load_safetensors_dir(ckpt)
    eng = LLMEngine(ref, tok, EngineConfig(max_num_seqs=8, max_model_len=512, max_batched_tokens=64,
                                           use_graphs=False))
    outs = eng.generate([apply_chat_template(m, tok) for m in msgs],
                        SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True))
    res["ref"] = [o.text for o in outs]
    with open(os.path.join(out_dir, "tp_serving.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def interleave_dp(iters):
    """One process replaying a DP=len(iters) job: each global batch = the ranks' micro-batches stacked."""
    while True:
        parts = [next(it) for it in iters]
        yield torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])


def full_sft_worker(rank, world, tp, port, out_dir):
    """Full-weight SFT at TP=tp x DP=world/tp. Every rank also replays the job in one process (TP=1, the DP
    ranks' micro-batches stacked) and compares its own shard of those weights with what it trained."""
    import json

    ctx = _init(rank, world, port, tp)
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext
    from generativeaiexamples_amd.training.data import batches, synthetic_rows
    from generativeaiexamples_amd.training.full import FullTrainer
    from generativeaiexamples_amd.training.trainer import TrainConfig

    cfg = LlamaConfig.tiny(num_layers=2, num_heads=4, num_kv_heads=2, head_dim=32, hidden_size=128,
                           intermediate_size=256)
    init = LlamaModel(cfg, device="cpu", dist_ctx=DistContext(), dtype=torch.float32).random_init(seed=5)
    sd0 = init.export_hf_state()
    m = LlamaModel(cfg, device="cpu", dist_ctx=ctx, dtype=torch.float32).load_hf_state(sd0)
    tok = small_byte_tokenizer(512)
    rows = synthetic_rows(64)
    dpn, dp = ctx.dp_size, ctx.dp_rank
    tcfg = dict(steps=3, global_batch=dpn, seq_len=64, lr=1e-3, warmup=1)
    tr = FullTrainer(m, tok, TrainConfig(micro_batch=1, **tcfg), batches(rows[dp::dpn], tok, 64, 1, seed=dp))
    hist = tr.train()
    one = LlamaModel(cfg, device="cpu", dist_ctx=DistContext(), dtype=torch.float32).load_hf_state(sd0)
    ref = FullTrainer(one, tok, TrainConfig(micro_batch=dpn, **tcfg),
                      interleave_dp([batches(rows[d::dpn], tok, 64, 1, seed=d) for d in range(dpn)]))
    ref_hist = ref.train()
    mine = LlamaModel(cfg, device="cpu", dist_ctx=ctx, dtype=torch.float32).load_hf_state(
        {k: v.detach() for k, v in one.export_hf_state().items()})
    err = max(float((m.w[k].detach() - mine.w[k]).abs().max()) for k in m.w)
    with open(os.path.join(out_dir, f"full_sft_{rank}.json"), "w") as f:
        json.dump({"loss": hist, "ref_loss": ref_hist, "max_err": err}, f)
    dist.barrier()
    dist.destroy_process_group()


def tp_linear_overlap_worker(rank, world, port, out_dir):
    """tp_linear_all_reduce (row-chunked GEMM + async all-reduce) == linear + all-reduce, and the TP Llama
    prefill with the overlapped path == the plain TP path."""
    ctx = _init(rank, world, port, world)
    from generativeaiexamples_amd import ops

    g = torch.Generator().manual_seed(1)
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(300, 64, generator=g).to(dt)  # this rank's K-shard of the activations
        w = torch.randn(48, 64, generator=g).to(dt)
        b = torch.randn(48, generator=g).to(dt) if rank == 0 else None
        got = ctx.tp_linear_all_reduce(x + rank, w * (rank + 1), b, chunks=3)
        want = ctx.tp_all_reduce(ops.linear(x + rank, w * (rank + 1), bias=b))
        res[str(dt)] = (got.float() - want.float()).abs().max().item()
    torch.save(res, os.path.join(out_dir, f"ovl_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def tp_graph_rehearsal_worker(rank, world, port, out_dir, shape="tiny"):
    """One-GPU rehearsal of a TP=world decode (every rank on cuda:0, gloo control plane): the multi-step
    decode graph holds only peer-memory collectives (custom all-reduce for the embedding / block-boundary
    reductions and ops.sample_tp's candidate exchange), is captured on every rank and replayed in lockstep
    through pipelined (chained) runs. Rank 0 checks every greedy token against the fp32 reference forward of
    the same weights (bf16 TP partial sums may flip a near-tie, after which the sequences legitimately
    diverge, so token-by-token equality with a TP=1 engine is not the criterion)."""
    import json
    import time as _time

    t_start = _time.monotonic()

    def progress(msg):  # per-rank timestamped progress (read by the test when a rank is late or hangs)
        with open(os.path.join(out_dir, f"tpg_progress_{rank}.txt"), "a") as f:
            f.write(f"{_time.monotonic() - t_start:8.3f}s {msg}\n")

    os.environ.update(GAI_SINGLE_DEVICE="1", GAI_CUSTOM_AR="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    # every rank's spin-waiting all-reduce kernel must be resident at once on the ONE shared GPU: one hardware
    # queue per process keeps 8 processes within the device's mapped queues (no time-sliced queue, whose
    # kernel would never meet its peers)
    one_gpu_rank_env(world)
    from generativeaiexamples_amd.parallel import dist as gdist

    ctx = gdist.init_distributed(tp_size=world, backend="gloo")
    progress(f"init pid {os.getpid()}")
    from generativeaiexamples_amd import ops
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer, small_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext

    err = None
    try:
        assert ctx.custom_ar is not None, "custom all-reduce not created"
        us = coresidency_probe(ctx.custom_ar, torch.device("cuda", 0), out_dir, "tpg", rank)
        progress(f"co-residency probe {us:.1f} us / all-reduce")
        if shape == "70b":  # Llama-3-70B layer widths (2 layers): real all-reduce message sizes, V / 8 sampler shards
            import dataclasses
            cfg = dataclasses.replace(LlamaConfig.llama3_70b(), num_layers=2, max_position=1024)
        else:
            cfg = LlamaConfig.tiny(num_heads=8, num_kv_heads=8, head_dim=64, hidden_size=512, intermediate_size=1024,
                                   vocab_size=4096)
        ref = LlamaModel(cfg, device="cuda", dist_ctx=DistContext()).random_init(17)
        m = LlamaModel(cfg, device="cuda", dist_ctx=ctx).load_hf_state(ref.export_hf_state())
        if rank != 0:
            del ref  # only the leader checks tokens against the fp32 reference
            torch.cuda.empty_cache()
        tok = small_byte_tokenizer(cfg.vocab_size) if cfg.vocab_size <= 4096 else llama3_byte_tokenizer(cfg.vocab_size)
        ecfg = dict(num_blocks=128, max_model_len=256, use_graphs=True, decode_steps=4, max_num_seqs=8,
                    graph_batch_sizes=(4, 8), prefix_cache=False, kv_memory_fraction=0.02)
        progress("model loaded")
        eng = LLMEngine(m, tok, EngineConfig(**ecfg))
        eng.capture_graphs(max_bs=8)
        progress(f"graphs captured {sorted(eng.multi_graphs)}")
        if not eng.leader:
            assert eng.follow() == "stop"
            progress("follower stopped")
        else:
            prompts = [list(range(11 + 3 * i, 11 + 3 * i + n)) for i, n in enumerate((9, 23, 40, 5, 17))]
            sp = SamplingParams(temperature=0.0, max_tokens=16, ignore_eos=True)
            tp = [eng.add_request(p_, sp) for p_ in prompts]
            while eng.has_work():
                eng.step()
                progress(f"step {eng.stats['steps']} graph_steps {eng.stats['graph_steps']} "
                         f"ar_err {int(ctx.custom_ar.err.item())}")
            stats = dict(eng.stats)
            eng.release_followers(stop=True)
            bad, total = [], 0
            for p, r in zip(prompts, tp):
                lg = ref.reference_forward(torch.tensor(p + r.output_ids[:-1]))[len(p) - 1:]
                for i, t in enumerate(r.output_ids):
                    total += 1
                    row = lg[i]
                    if float(row[t]) < float(row.max()) - 0.02 * max(1.0, float(row.abs().max())):
                        bad.append((i, t, int(row.argmax())))
            with open(os.path.join(out_dir, "tpg.json"), "w") as f:
                json.dump({"bad": bad, "total": total, "stats": stats, "multi_graphs": sorted(eng.multi_graphs),
                           "flags": int(ops.tp_sample_flags(m.device))}, f)
    except Exception:  # noqa: BLE001
        import traceback
        err = traceback.format_exc()
        with open(os.path.join(out_dir, f"tpg_err_{rank}.txt"), "w") as f:
            f.write(err)
    finally:
        gdist.shutdown()
    if err:
        raise SystemExit(1)


def ep_engine_worker(rank, world, port, out_dir):
    """Data-parallel attention + expert parallelism (MixtralModel ep_group, all-to-all token exchange): each
    rank serves its OWN requests (different counts and lengths, so ranks run dummy lockstep steps) with 8 / world
    experts; its greedy tokens must equal a single-process Mixtral's on the same prompts (fp32)."""
    import json

    ctx = _init(rank, world, port, 1)
    import torch.distributed as dist

    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models.mixtral import MixtralConfig, MixtralModel
    from generativeaiexamples_amd.parallel.dist import DistContext

    cfg = MixtralConfig.tiny_moe(num_experts=8)
    ref = MixtralModel(cfg, device="cpu", dtype=torch.float32, dist_ctx=DistContext()).random_init(3)
    m = MixtralModel(cfg, device="cpu", dtype=torch.float32, dist_ctx=ctx, ep_group=dist.group.WORLD)
    with torch.no_grad():
        for k, t in m.w.items():
            src = ref.w[k]
            if k.endswith("w13") or k.endswith("w2"):
                src = src[m.e_start:m.e_start + m.e_local]
            t.copy_(src)
    tok = small_byte_tokenizer(512)
    prompts = [list(range(5 + 7 * rank + 3 * i, 5 + 7 * rank + 3 * i + 6 + 9 * ((i + rank) % 3))) for i in range(rank + 1)]
    sp = SamplingParams(temperature=0.0, max_tokens=5 + 3 * rank, ignore_eos=True)
    ecfg = dict(num_blocks=96, max_model_len=256, use_graphs=False, max_num_seqs=8, max_batched_tokens=64,
                prefill_chunk=32, prefix_cache=False)
    eng = LLMEngine(m, tok, EngineConfig(**ecfg))
    ep = [r.output_ids for r in eng.generate(prompts, sp)]
    one = [r.output_ids for r in LLMEngine(ref, tok, EngineConfig(**ecfg)).generate(prompts, sp)]
    with open(os.path.join(out_dir, f"ep_{rank}.json"), "w") as f:
        json.dump({"ep": ep, "ref": one, "e_local": m.e_local, "steps": eng.stats["steps"]}, f)
    dist.barrier()
    dist.destroy_process_group()


ROUTER_TIE = 0.05  # router-logit gap (k-th vs (k+1)-th expert) below which bf16 routing may legitimately differ


def moe_greedy_check(model, prompts, outputs, tie=ROUTER_TIE, device="cpu"):
    """Greedy MoE tokens vs the fp32 oracle: a token is consistent when its fp32 logit is within 2 % of the row's
    max (a bf16 near-tie). A miss where some token of the prefix had a near-tie top-k routing in some layer (the bf16
    engine may have picked the other expert there) is reported apart, and the rest of that request is not judged
    against the oracle. -> (bad, router_ties, total)."""
    bad, ties, total = [], [], 0
    for p, out in zip(prompts, outputs):
        margins = []
        lg = model.reference_forward(torch.tensor(p + out[:-1]), router_margin=margins, device=device)
        mg = margins[0]
        for i, t in enumerate(out):
            total += 1
            row = lg[len(p) - 1 + i]
            tol = 0.02 * max(1.0, float(row.abs().max()))
            if float(row[t]) < float(row.max()) - tol:
                # a near-tie routing of this token OR of any earlier one (its keys / values then differ from the
                # oracle's for every later position of the request)
                m = float(mg[: len(p) + i].min())
                rec = (i, t, int(row.argmax()), round(float(row.max() - row[t]), 4), round(tol, 4), round(m, 4))
                if m < tie:
                    ties.append(rec)
                    total += len(out) - i - 1  # the rest of this request follows a legitimately different route
                    break
                bad.append(rec)
    return bad, ties, total


def moe_divergence_explained(model, prompt, a, b, tie=ROUTER_TIE, device="cpu"):
    """Two greedy continuations ``a`` / ``b`` of one prompt (EP engine vs single-rank engine) may part only where
    bf16 can legitimately decide either way: at their first differing position the fp32 oracle has the two tokens
    within a near-tie, or some token of the shared prefix has a near-tie top-k routing. -> (explained, detail)."""
    j = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), None)
    if j is None:
        return len(a) == len(b), {"len": (len(a), len(b))}
    margins = []
    lg = model.reference_forward(torch.tensor(prompt + a[:j]), router_margin=margins, device=device)
    row = lg[-1]
    tol = 0.02 * max(1.0, float(row.abs().max()))
    gap = abs(float(row[a[j]]) - float(row[b[j]]))
    m = float(margins[0].min())
    return bool(gap <= tol or m < tie), {"pos": j, "tokens": (a[j], b[j]), "logit_gap": round(gap, 4),
                                        "tol": round(tol, 4), "router_margin": round(m, 4)}


def ep_gpu_rehearsal_worker(rank, world, port, out_dir, shape="tiny"):
    """One-GPU rehearsal of Mixtral expert parallelism (VERDICT r3 "next" #4): ``world`` ranks share cuda:0 over a
    gloo control plane; each owns 8 / world experts and serves its OWN requests (different counts and lengths:
    idle ranks replay padding-only graphs). Prefill steps use the exact-count exchange, decode steps run as
    captured HIP graphs whose token exchanges are the peer-memory one-shot all-to-all (native EP pack / combine
    kernels around it). Every greedy token must be the fp32 reference argmax of its prefix up to a bf16 near-tie."""
    import json
    import time as _time

    t_start = _time.monotonic()

    def progress(msg):
        with open(os.path.join(out_dir, f"ep_progress_{rank}.txt"), "a") as f:
            f.write(f"{_time.monotonic() - t_start:8.3f}s {msg}\n")

    os.environ.update(GAI_SINGLE_DEVICE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    one_gpu_rank_env(world)  # as the TP rehearsal: every rank's spin-waiting exchange resident at once
    from generativeaiexamples_amd.parallel import dist as gdist

    ctx = gdist.init_distributed(tp_size=1, backend="gloo")
    progress(f"init pid {os.getpid()}")
    import torch.distributed as dist

    from generativeaiexamples_amd import ops
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models.mixtral import MixtralConfig, MixtralModel
    from generativeaiexamples_amd.parallel.dist import DistContext

    err = None
    try:
        if shape == "mixtral":  # Mixtral-8x7B layer widths (2 layers): d 4096, 8 experts of FFN 14336, V 32000
            import dataclasses
            cfg = dataclasses.replace(MixtralConfig.mixtral_8x7b(), num_layers=2, max_position=1024)
        else:
            cfg = MixtralConfig.tiny_moe(num_experts=8, hidden_size=512, intermediate_size=512, num_heads=8,
                                         num_kv_heads=4, head_dim=64, vocab_size=4096)
        ref = MixtralModel(cfg, device="cuda", dist_ctx=DistContext()).random_init(3)
        if shape == "mixtral":
            # random routers at d = 4096 put the 2nd and 3rd expert within bf16 noise for a few % of tokens per layer;
            # a trained router is far more decisive - scale the logits so near-ties stay rare (the exchange under
            # test is unaffected; ties are still detected and reported by the oracle)
            with torch.no_grad():
                for i in range(cfg.num_layers):
                    ref.w[f"l{i}.router"].mul_(8.0)
        m = MixtralModel(cfg, device="cuda", dist_ctx=ctx, ep_group=dist.group.WORLD)
        with torch.no_grad():
            for k, t in m.w.items():
                src = ref.w[k]
                if k.endswith("w13") or k.endswith("w2"):
                    src = src[m.e_start:m.e_start + m.e_local]
                t.copy_(src)
        assert m.ep_xchg is not None, "peer-memory all-to-all not created"
        us = coresidency_probe(m.ep_xchg, m.device, out_dir, "epg", rank)
        progress(f"co-residency probe {us:.1f} us / all-reduce")
        tok = small_byte_tokenizer(min(cfg.vocab_size, 4096))
        graphs = os.environ.get("GAI_EP_REHEARSE_GRAPHS", "1") == "1"  # "0": eager decode (A/B of a failure)
        ecfg = dict(num_blocks=160, max_model_len=256, use_graphs=graphs, max_num_seqs=8, max_batched_tokens=64,
                    prefill_chunk=32, prefix_cache=False, graph_batch_sizes=(1, 2, 4, 8), kv_memory_fraction=0.02)
        eng = LLMEngine(m, tok, EngineConfig(**ecfg))
        if graphs:
            eng.capture_graphs(max_bs=8)
        progress(f"graphs captured {sorted(eng.graphs)}")
        n_req = 1 + 2 * rank  # ranks carry different loads: idle ranks replay padding-only graphs
        prompts = [list(range(11 + 5 * rank + 3 * i, 11 + 5 * rank + 3 * i + 7 + 9 * ((i + rank) % 3)))
                   for i in range(n_req)]
        sp = SamplingParams(temperature=0.0, max_tokens=6 + 4 * rank, ignore_eos=True)
        reqs = [eng.add_request(p_, sp) for p_ in prompts]
        while True:
            busy = int(eng.has_work())
            if not eng._ep_agree([busy])[0]:  # lockstep until every rank is done
                break
            eng.step()
            progress(f"step {eng.stats['steps']} graph_steps {eng.stats['graph_steps']} err {int(m.ep_xchg.err.item())}")
        odev = "cuda" if shape == "mixtral" else "cpu"  # full-width fp32 oracle on the GPU (plain torch ops)
        bad, ties, total = moe_greedy_check(ref, prompts, [r.output_ids for r in reqs], device=odev)
        # the same requests on a single-rank engine over the full model (no exchange), for the record: its decode
        # batches have no cross-rank padding, so the grouped GEMMs pick other tile shapes (other fp32 summation
        # orders) and a near-tie can resolve differently; both runs are judged by the fp32 oracle above
        ref_eng = LLMEngine(ref, tok, EngineConfig(**ecfg))
        ref_reqs = [ref_eng.add_request(p_, sp) for p_ in prompts]
        while ref_eng.has_work():
            ref_eng.step()
        differ, unexplained = [], []
        for i, (a, b) in enumerate(zip(reqs, ref_reqs)):
            if a.output_ids != b.output_ids:
                ok, det = moe_divergence_explained(ref, prompts[i], a.output_ids, b.output_ids, device=odev)
                (differ if ok else unexplained).append((i, det))
        with open(os.path.join(out_dir, f"epg_{rank}.json"), "w") as f:
            json.dump({"bad": bad, "ties": ties, "total": total, "differ_from_single_rank": differ,
                       "differ_unexplained": unexplained, "stats": dict(eng.stats), "graphs": sorted(eng.graphs),
                       "lens": [len(r.output_ids) for r in reqs], "err": int(m.ep_xchg.err.item())}, f)
    except Exception:  # noqa: BLE001
        import traceback
        err = traceback.format_exc()
        with open(os.path.join(out_dir, f"epg_err_{rank}.txt"), "w") as f:
            f.write(err)
    finally:
        gdist.shutdown()
    if err:
        raise SystemExit(1)
