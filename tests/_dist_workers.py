"""Worker bodies for the multi-process (gloo, 127.0.0.1) distributed tests."""
import os

import torch
import torch.distributed as dist


def _init(rank, world, port, tp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from generativeaiexamples_amd.parallel import dist as gdist

    return gdist.init_distributed(tp_size=tp, backend="gloo")


def tp_llama_worker(rank, world, port, out_dir):
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
    rows, eid, plan = ep.dispatch(x, ids, w, E, None)
    y = ep.local_experts(rows, eid, w13[rank * e_local:(rank + 1) * e_local], w2[rank * e_local:(rank + 1) * e_local])
    out = ep.combine(y, w, plan, None)
    # single-process oracle with all experts
    a_rows, offs, pos = ops.moe_dispatch(ids, E)
    h1 = ops.moe_gemm(x, a_rows, w13, offs, x.shape[0] * k, True)
    yy = ops.moe_gemm(h1, None, w2, offs, x.shape[0] * k, False)
    exp = ops.moe_combine(yy, pos, w)
    torch.save({"out": out.float(), "exp": exp.float()}, os.path.join(out_dir, f"ep_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def sharded_index_worker(rank, world, port, out_dir):
    _init(rank, world, port, 1)
    from generativeaiexamples_amd.index.hbm_index import HBMIndex
    from generativeaiexamples_amd.index.sharded import ShardedIndex

    g = torch.Generator().manual_seed(0)
    full = torch.nn.functional.normalize(torch.randn(2 * 300, 32, generator=g), dim=-1)
    queries = torch.nn.functional.normalize(torch.randn(2 * 5, 32, generator=g), dim=-1)
    shard = full[rank * 300:(rank + 1) * 300]
    idx = HBMIndex(32, "cosine", device="cpu", capacity=16)
    idx.add(shard)
    si = ShardedIndex(idx)
    my_q = queries[rank * 5:(rank + 1) * 5]
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
