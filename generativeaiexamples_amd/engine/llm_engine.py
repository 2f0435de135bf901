"""Generator engine: continuous batching over the native scheduler, paged KV, HIP-graph decode.

Replaces the LLM NIM (TRT-LLM / vLLM inside ``nvcr.io/nim/meta/llama3-8b-instruct``, SURVEY S1,
call stack §3.3 steps 3.1.2: tokenize -> prefill -> decode loop -> detokenize -> SSE delta).

One :meth:`LLMEngine.step`:
  1. ``_rt.Scheduler.schedule()`` (C++) picks decodes + prefill chunks under the token budget and
     flattens them into int32 arrays (token ids, positions, KV slots, varlen metadata);
  2. the arrays go to the GPU in ONE pinned host->device copy;
  3. the model runs (decode-only steps replay a captured HIP graph for the padded batch size);
  4. the gfx950 sampler draws one token per finished-prompt / decode row;
  5. tokens come back to the host, stop conditions (EOS, stop ids, stop strings, max_tokens) are
     applied and text deltas are produced by the incremental detokenizer.

Multi-step decode (``EngineConfig.decode_steps``): once every running sequence is decoding and none
is waiting, the scheduler reserves KV pages for K tokens per sequence and ONE captured HIP graph runs
K x (forward -> sample -> ``decode_advance``), feeding each sampled token back as the next input on
the device. The host syncs once per K tokens instead of once per token, so the per-token Python /
launch / H2D cost (~1 ms per step at batch 64) leaves the decode loop; tokens past a stop condition
are discarded.
"""
from __future__ import annotations

import itertools
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..models.common import ForwardBatch
from .kv_cache import KVCache, cache_dtype
from .sampling import SamplingBatch, SamplingParams
from .staging import HostStager
from ..utils.graphs import hip_graph_capture
from ..utils.profiling import roctx_range
from .tokenizer import IncrementalDetokenizer, Tokenizer


def _rt():
    from .. import _rt as m  # native runtime (C++), built by generativeaiexamples_amd._build

    return m


@dataclass
class EngineConfig:
    max_num_seqs: int = 256
    max_batched_tokens: int = 16384
    max_model_len: int = 8192
    prefill_chunk: int = 16384
    num_blocks: Optional[int] = None
    kv_memory_fraction: float = 0.80      # of the HBM left after weights
    kv_memory_bytes: Optional[int] = None
    prefix_cache: bool = True
    use_graphs: bool = True
    # keep MFMA-fragment-shuffled copies of the decode projections (ops.preshuffle_weight, see
    # LlamaModel.DECODE_PROJECTIONS): every decode weight stream then reads whole 128-B lines
    # (non-temporal), +9 % decode / +4.9 % headline on the same box (profiles/r3/psw_ab) for a second copy of
    # the projection weights (17 GB for Llama-3-8B: 6 % of one MI355X's 288 GB)
    decode_preshuffle: bool = True
    # "fragment": the decode projections are stored ONCE, in MFMA fragment order (rewritten in place; the prefill
    # GEMMs, decode GEMMs and GEMV all read that layout), instead of row-major weights plus a fragment-ordered copy
    # ("dual"). GAI_WEIGHT_LAYOUT overrides (same-box A/B).
    weight_layout: str = "fragment"
    graph_batch_sizes: Sequence[int] = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256)
    # multi-step decode: when every running sequence is decoding (nothing waiting), run this many
    # decode steps in ONE captured HIP graph (forward -> sample -> feed the token back, on device)
    # and return to the host once per run. 1 disables it.
    decode_steps: int = 8
    # "auto" = the model dtype; "fp8" = OCP e4m3fn KV cache (twice the cached tokens per GB, half the decode
    # attention bytes; static per-layer scales kv_scale), for models whose attention path supports it
    kv_cache_dtype: str = "auto"
    kv_scale: float = 1.0


@dataclass
class Request:
    request_id: str
    prompt_ids: List[int]
    params: SamplingParams
    seq_id: int
    detok: IncrementalDetokenizer
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    output_ids: List[int] = field(default_factory=list)
    finished: bool = False
    finish_reason: Optional[str] = None
    seed: int = 0
    token_counts: Dict[int, int] = field(default_factory=dict)
    lora_slot: int = 0
    max_new: int = 0
    matcher: Any = None  # constrained decoding (engine/guided.py): this request's grammar state
    mask_empty: bool = False  # the grammar allows no token within the remaining budget

    @property
    def text(self) -> str:
        return self.detok.text

    @property
    def ttft(self) -> Optional[float]:
        return None if self.first_token_time is None else self.first_token_time - self.arrival


@dataclass
class RequestOutput:
    request_id: str
    token_id: int
    delta: str
    finished: bool
    finish_reason: Optional[str] = None


@dataclass
class _Run:
    """A K-step decode graph run enqueued on the device whose sampled tokens are not processed yet."""
    ids: List[int]            # sequence ids in row order
    reqs: List[Request]
    K: int
    n: int
    chained: bool             # first input fed on the device from the previous run's last token
    base: List[int]           # absolute position of each row's first input token
    host: Any                 # [K, bucket] int32 tokens (pinned; valid once `done` has completed)
    done: Any = None          # device event after the tokens' D2H copy (None: already synchronous)


@dataclass
class _Single:
    """A one-token step enqueued on the device whose sampled tokens are not processed yet."""
    seq_order: List[int]
    reqs: List[Any]
    n: int
    host: Any                 # sampled tokens (pinned buffer view, valid once `done` completed) or a list
    done: Any = None


class LLMEngine:
    def __init__(self, model, tokenizer: Tokenizer, cfg: EngineConfig | None = None):
        self.model, self.tok = model, tokenizer
        self.cfg = cfg = cfg or EngineConfig()
        self.device = model.device
        mc = model.cfg
        cfg.max_model_len = min(cfg.max_model_len, mc.max_position)
        self.max_blocks_per_seq = (cfg.max_model_len + ops.BLOCK - 1) // ops.BLOCK
        psw = os.environ.get("GAI_DECODE_PSW")  # "1" / "0" overrides the config (same-box A/B)
        if (self.device.type == "cuda" and (cfg.decode_preshuffle if psw is None else psw == "1")
                and hasattr(model, "preshuffle_decode_weights")):
            # before KV sizing: the fragment copies are resident; at most 20 % of the device's HBM
            total = torch.cuda.get_device_properties(self.device).total_memory
            layout = os.environ.get("GAI_WEIGHT_LAYOUT", cfg.weight_layout)
            if layout not in ("fragment", "dual"):
                raise ValueError(f"weight_layout {layout!r}: expected 'fragment' or 'dual'")
            model.preshuffle_decode_weights(budget_bytes=int(0.2 * total), in_place=layout == "fragment")
        # tensor parallel: rank 0 of the TP group plans every step, the other members execute its plans
        ctx = getattr(model, "ctx", None)
        self.tp_size = ctx.tp_size if ctx is not None else 1
        self.leader = self.tp_size == 1 or ctx.tp_rank == 0
        # multi-step decode graphs hold only peer-memory collectives when the TP group has the custom all-reduce
        # (the embedding / block-boundary all-reduces and sample_tp's candidate exchange), so they are captured
        # even over a gloo control plane (one-GPU TP rehearsal, GAI_SINGLE_DEVICE=1)
        self.multi_graphs_ok = cfg.use_graphs and (self.tp_size == 1 or ctx.backend == "nccl"
                                                   or getattr(ctx, "custom_ar", None) is not None)
        if self.tp_size > 1 and self.device.type == "cuda" and ctx.backend != "nccl":
            cfg.use_graphs = False  # host (gloo) collectives, e.g. a one-GPU TP rehearsal, are not capturable
        if self.tp_size > 1 and hasattr(model, "register_request"):
            raise NotImplementedError(f"{mc.name}: per-request model state is not replicated to TP followers")
        self.kv_dtype = cache_dtype(cfg.kv_cache_dtype, model.dtype)
        if self.kv_dtype == torch.float8_e4m3fn and not getattr(model, "supports_fp8_kv", False):
            raise ValueError(f"{mc.name}: the fp8 KV cache is not supported by this model's attention path")
        nb = cfg.num_blocks or self._blocks_from_memory()
        if self.tp_size > 1:  # every rank's cache must hold the leader's block ids: agree on the minimum
            import torch.distributed as dist
            t = torch.tensor([nb], dtype=torch.int64,
                             device=self.device if ctx.backend == "nccl" else torch.device("cpu"))
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.tp_group)
            nb = int(t.item())
        # one extra block, never handed out, is the scratch page of padded graph rows
        # models with non-KV layers (cross-attention) report how many layers own a paged KV cache
        self.kv = KVCache(self._kv_layers(), nb + 1, model.hkv, mc.head_dim, self.device, self.kv_dtype,
                          k_scale=cfg.kv_scale, v_scale=cfg.kv_scale)
        self.pad_block = nb
        self.sched = _rt().Scheduler(nb, cfg.max_num_seqs, cfg.max_batched_tokens, cfg.max_model_len,
                                     cfg.prefix_cache, cfg.prefill_chunk)
        self.decode_ws = None
        if self.device.type == "cuda":
            self.decode_ws = ops.DecodeWorkspace(max(cfg.max_num_seqs, max(cfg.graph_batch_sizes)), model.hq,
                                                 mc.head_dim, max(cfg.max_model_len,
                                                                  getattr(model, "max_cross_tokens", 0)),
                                                 self.device)
        # two staging banks used by alternate launches: a pipelined run's H2D copies may still be queued
        # behind the run in flight when the host stages the next one (HostStager.reset waits on the fence)
        self.stagers = [HostStager(self.device), HostStager(self.device)]
        self.stager = self.stagers[0]
        self._pending: Optional[_Run] = None  # multi-step run enqueued, tokens not processed yet
        self._launches = 0
        self._tok_host = None  # 2 pinned [K * max bucket] int32 token buffers (alternate launches)
        self._single_host = None  # 2 pinned token buffers of one-token steps (alternate launches)
        # schedule + enqueue the next batch while a one-token step is still on the device (prefill chunks
        # back to back: the host's planning / launches overlap the GPU instead of following a sync)
        self._lookahead = os.environ.get("GAI_LOOKAHEAD", "1") == "1"
        self._pipeline = os.environ.get("GAI_PIPELINE", "1") == "1"  # chained multi-step runs (A/B switch)
        self._masks = None  # guided-decoding mask builder (lazy)
        self._timing = os.environ.get("GAI_STEP_TIMING") == "1"
        # GAI_HOST_TIMELINE=1: (event, t_start, t_end) host timestamps of the pipelined decode (chain / complete /
        # non-chained launches), no synchronisation added - for finding host gaps between graph runs
        self.host_timeline: Optional[list] = [] if os.environ.get("GAI_HOST_TIMELINE") == "1" else None
        self.phase_ms: Dict[str, float] = {}
        self._t_mark = 0.0
        self.requests: Dict[int, Request] = {}
        self.by_rid: Dict[str, Request] = {}
        self._ids = itertools.count(1)
        self.step_count = 0
        self.graphs: Dict[int, tuple] = {}
        self.multi_graphs: Dict[int, tuple] = {}
        self.lock = threading.RLock()
        self.stats = dict(prefill_tokens=0, decode_tokens=0, steps=0, graph_steps=0, multi_step_runs=0,
                          chained_runs=0)
        self.eos = set(mc.eos_token_ids) | set(getattr(tokenizer, "eos_ids", ()) or ())
        self.chan = None
        if self.tp_size > 1:
            from ..parallel.step_channel import StepChannel
            self.chan = StepChannel(ctx)
        # expert parallelism with data-parallel attention (MixtralModel ep_group): every rank runs its own
        # requests, but each MoE layer is an all-to-all over the group, so the ranks step in LOCKSTEP: one
        # small all-reduce per step agrees on the largest token count (the padded exchange's capacity) and
        # on whether anyone prefills; a rank with nothing scheduled runs a one-token dummy forward
        self.ep_group = getattr(model, "ep_group", None)
        self._ep_bucket: Optional[int] = None  # EP lockstep: the graph bucket every rank replays this step
        if self.ep_group is not None:
            import torch.distributed as dist
            # single-step decode graphs when the step's exchanges are capturable: RCCL, or the peer-memory
            # all-to-all (model.ep_xchg) over any control plane; every rank replays the bucket of the largest
            # per-rank batch, so all ranks exchange slabs of one capacity
            cfg.use_graphs = cfg.use_graphs and self.device.type == "cuda" and (
                dist.get_backend(self.ep_group) == "nccl" or getattr(model, "ep_xchg", None) is not None)
            self.multi_graphs_ok = False
            cfg.decode_steps = 1

    # ------------------------------------------------------------------ memory
    def _kv_layers(self) -> int:
        return getattr(self.model, "num_kv_layers", self.model.cfg.num_layers)

    def _blocks_from_memory(self) -> int:
        mc = self.model.cfg
        if self.cfg.kv_memory_bytes:
            nbytes = self.cfg.kv_memory_bytes
        elif self.device.type == "cuda":
            free, _total = torch.cuda.mem_get_info(self.device)
            frac = self.cfg.kv_memory_fraction
            if os.environ.get("GAI_SINGLE_DEVICE") == "1":  # rehearsal: every rank shares this one GPU
                frac /= max(1, int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1"))))
            nbytes = int(free * frac)
        else:
            nbytes = 256 << 20
        nb = KVCache.blocks_for_memory(nbytes, self._kv_layers(), self.model.hkv, mc.head_dim, self.kv_dtype)
        return max(nb, 2 * self.max_blocks_per_seq)

    # ------------------------------------------------------------------ requests
    def add_request(self, prompt_ids: List[int], params: SamplingParams | None = None,
                    request_id: Optional[str] = None, images: Optional[list] = None,
                    lora: Optional[str] = None) -> Request:
        """images: inputs for a multimodal model (encoded once here by ``model.register_request``);
        lora: name of an adapter registered with ``model.add_lora`` (multi-LoRA serving)."""
        params = params or SamplingParams()
        if params.resume_ids:
            prompt_ids = list(prompt_ids) + list(params.resume_ids)
        with self.lock:
            sid = next(self._ids)
            rid = request_id or f"req-{sid}"
            max_new = max(0, min(params.max_tokens, self.cfg.max_model_len - len(prompt_ids)))
            if len(prompt_ids) >= self.cfg.max_model_len:
                # keep the tail (reference truncates retrieved context the same way: truncate="END")
                prompt_ids = prompt_ids[-(self.cfg.max_model_len - 1):]
                max_new = 1
            req = Request(rid, list(prompt_ids), params, sid, IncrementalDetokenizer(self.tok, params.stop),
                          seed=params.seed if params.seed is not None else (sid * 7919) & 0x7FFFFFFF)
            req.max_new = max_new
            if params.guided is not None:
                req.matcher = params.guided.matcher()
                for t in params.resume_ids:
                    req.matcher.advance(int(t))
            if params.resume_ids:
                req.detok.prime(params.resume_ids, params.resume_sent_chars)
            for t in params.resume_ids:
                req.token_counts[t] = req.token_counts.get(t, 0) + 1
            if lora:
                req.lora_slot = self.model.lora_slot(lora)
            self.requests[sid] = req
            self.by_rid[rid] = req
            if images:
                if not hasattr(self.model, "register_request"):
                    raise ValueError(f"{self.model.cfg.name} does not accept image inputs")
                self.model.register_request(sid, images, prompt_ids=req.prompt_ids)
            if max_new == 0:
                self._release(sid)
                req.finished, req.finish_reason = True, "length"
                return req
            self.sched.add(sid, req.prompt_ids, max_new)
            return req

    def abort(self, request_id: str) -> bool:
        with self.lock:
            req = self.by_rid.pop(request_id, None)
            if req is None:
                return False
            self.sched.abort(req.seq_id)
            self.requests.pop(req.seq_id, None)
            self._release(req.seq_id)
            req.finished, req.finish_reason = True, "abort"
            return True

    def add_lora(self, name: str, adapter) -> int:
        """Register a LoRA adapter (object or directory) for per-request selection. Captured decode graphs
        are dropped and re-captured lazily so they include the new adapter's deltas."""
        with self.lock:
            if self.chan is not None and self.leader:
                if not isinstance(adapter, str):
                    raise ValueError("tensor-parallel engines load LoRA adapters by path (every rank loads it)")
                self.chan.send({"op": "call", "fn": "add_lora", "args": [name, adapter]})
            slot = self.model.add_lora(name, adapter)
            self.graphs.clear()
            return slot

    def _release(self, sid: int):
        if hasattr(self.model, "release_request"):
            self.model.release_request(sid)

    def has_work(self) -> bool:
        """EP lockstep engines: a collective over the EP group (True while ANY rank has work), so every rank
        calls it, and step(), the same number of times."""
        local = self._pending is not None or self.sched.has_work()
        if self.ep_group is None:
            return local
        return bool(self._ep_agree([int(local)])[0])

    def _ep_agree(self, vals: List[int]) -> List[int]:
        import torch.distributed as dist

        dev = self.device if dist.get_backend(self.ep_group) == "nccl" else torch.device("cpu")
        t = torch.tensor(vals, dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ep_group)
        return [int(v) for v in t.tolist()]

    def _ep_idle_graph(self, t_max: int) -> None:
        """A rank with nothing scheduled replays the step's bucket graph with every row padding (scratch page,
        ctx 1): it joins the same captured all-to-alls as its busy peers."""
        z = np.zeros(0, np.int32)
        plan = dict(op="graph", n=0, arr=[z, z, z, z, np.zeros((0, 1), np.int32)], seq_ids=[])
        self._bank()
        self._run_graph(plan)
        self.stager.fence()
        self._step_done()

    def _ep_dummy_forward(self) -> None:
        """One decode row on the scratch page: keeps this rank in the step's all-to-alls."""
        d = self.device
        i32 = dict(dtype=torch.int32, device=d)
        fb = ForwardBatch(token_ids=torch.zeros(1, **i32), positions=torch.zeros(1, **i32),
                          slots=torch.full((1,), self.pad_block * ops.BLOCK, **i32), num_prefill_tokens=0,
                          decode_ctx=torch.ones(1, **i32), decode_block_tables=torch.full((1, 1), self.pad_block, **i32),
                          max_decode_ctx=1, sample_rows=None)
        self.model.forward(fb, self.kv, self.decode_ws)
        self._step_done()

    # ------------------------------------------------------------------ batch construction
    def _to_device(self, arrays: List[np.ndarray]) -> List[torch.Tensor]:
        """Stage index / parameter arrays. int32, float32 and int64 keep their dtype (sampling temperature,
        top_p and 64-bit seeds must not be truncated); any other integer dtype is narrowed to int32."""
        out = []
        for a in arrays:
            a = np.asarray(a)
            if a.dtype not in (np.int32, np.float32, np.int64):
                a = a.astype(np.float32 if a.dtype.kind == "f" else np.int32)
            out.append(a)
        return self.stager.stage(out)

    # ------------------------------------------------------------------ step plans
    # A step is planned on the TP leader (scheduler decisions, sampling parameters, KV pages) and executed
    # from the plan on every rank: the plan is a dict of numpy arrays and plain values, published unchanged
    # to the follower ranks (parallel/step_channel.py) when the model is tensor-parallel.
    def _plan_eager(self, b) -> dict:
        P = b.num_prefill_tokens
        samples = b.prefill_samples
        cu = b.cu_q
        rows = []
        for i, sid in enumerate(b.prefill_seq_ids):
            if samples[i]:
                rows.append(int(cu[i + 1]) - 1)
        nd = len(b.decode_seq_ids)
        rows += range(P, P + nd)
        arrs = [b.token_ids, b.positions, b.slots, cu, b.prefill_ctx, b.prefill_block_tables, b.decode_ctx,
                b.decode_block_tables, np.asarray(rows, dtype=np.int32)]
        if P > 0:
            rpt = ops.prefill_rows_per_tile(self.model.hq, self.model.hkv, self.model.cfg.head_dim)
            arrs.append(ops.prefill_tile_list(b.prefill_qlen, rpt, b.prefill_ctx))
        plan = dict(op="eager", P=int(P), arr=arrs, qlen=[int(x) for x in b.prefill_qlen],
                    pctx=[int(x) for x in b.prefill_ctx], max_dctx=int(b.decode_ctx.max()) if nd else 0,
                    seq_ids=[int(x) for x in b.prefill_seq_ids] + [int(x) for x in b.decode_seq_ids],
                    pseq=[int(x) for x, smp in zip(b.prefill_seq_ids, samples) if smp])
        if getattr(self.model, "lora_names", None):
            per_seq = [self._slot(s) for s in plan["seq_ids"]]
            qlen = list(b.prefill_qlen) + [1] * nd
            plan["lora"] = np.repeat(np.asarray(per_seq, np.int32), qlen)
        return plan

    def _batch_from_plan(self, plan: dict) -> ForwardBatch:
        P = plan["P"]
        dev = self._to_device(plan["arr"] + ([plan["lora"]] if plan.get("lora") is not None else []))
        fb = ForwardBatch(token_ids=dev[0], positions=dev[1], slots=dev[2], num_prefill_tokens=P)
        if P > 0:
            fb.cu_q, fb.prefill_ctx, fb.prefill_block_tables = dev[3], dev[4], dev[5]
            fb.prefill_qlen = list(plan["qlen"])
            fb.prefill_ctx_host = list(plan["pctx"])
            fb.prefill_tiles = dev[9].reshape(-1)
        if plan["max_dctx"]:
            fb.decode_ctx, fb.decode_block_tables = dev[6], dev[7]
            fb.max_decode_ctx = plan["max_dctx"]
        fb.sample_rows = dev[8].long()
        fb.seq_ids = list(plan["seq_ids"])
        if plan.get("lora") is not None:
            fb.lora_slots = dev[-1]
        if hasattr(self.model, "prepare_batch"):
            self.model.prepare_batch(fb)
        return fb

    def _make_batch(self, b) -> tuple:
        """(ForwardBatch, sampled sequence ids) of a StepBatch, built through the eager plan (tests, tools)."""
        plan = self._plan_eager(b)
        return self._batch_from_plan(plan), plan["pseq"] + [int(x) for x in b.decode_seq_ids]

    def _publish(self, plan: dict) -> None:
        if self.chan is not None:
            self.chan.send(plan)

    def _step_done(self) -> None:
        """End of a step on every rank: (followers) wait for the step's GPU work so the staging buffers can
        be reused, then poll the custom all-reduce's error word (RankFailure on a missed peer). Expert-parallel
        ranks poll their peer-memory all-to-all's error word the same way: a peer that died or fell
        out of lockstep makes the exchange give up after its bounded spin with stale slot data, so the step's
        tokens are invalid; the exchange is retired (later exchanges go to RCCL, its captured graphs are
        dropped) and RankFailure is raised."""
        if self.tp_size > 1:
            if not self.leader and self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            self.model.ctx.check_comm()
        xchg = getattr(self.model, "ep_xchg", None) if self.ep_group is not None else None
        if xchg is not None:
            from ..parallel.fault import RankFailure

            if self.device.type == "cuda":  # EP steps are host-synchronous already (lockstep agreement)
                torch.cuda.current_stream(self.device).synchronize()
            try:
                xchg.check()
            except RankFailure:
                import torch.distributed as dist

                self.model.ep_xchg = None
                self.graphs.clear()
                self.multi_graphs.clear()
                if dist.get_backend(self.ep_group) != "nccl":  # the fallback exchange is not capturable
                    self.cfg.use_graphs = False
                raise

    # ------------------------------------------------------------------ HIP graphs (decode)
    def _slot(self, sid: int) -> int:
        r = self.requests.get(sid)
        return r.lora_slot if r is not None else 0

    def _graph_bucket(self, n: int) -> Optional[int]:
        for s in self.cfg.graph_batch_sizes:
            if s >= n:
                return s
        return None

    def _capture(self, bs: int):
        d = self.device
        ids = torch.zeros(bs, dtype=torch.int32, device=d)
        pos = torch.zeros(bs, dtype=torch.int32, device=d)
        slots = torch.full((bs,), self.pad_block * ops.BLOCK, dtype=torch.int32, device=d)
        ctx = torch.ones(bs, dtype=torch.int32, device=d)
        bt = torch.full((bs, self.max_blocks_per_seq), self.pad_block, dtype=torch.int32, device=d)
        fb = ForwardBatch(token_ids=ids, positions=pos, slots=slots, num_prefill_tokens=0, decode_ctx=ctx,
                          decode_block_tables=bt, max_decode_ctx=self.cfg.max_model_len, sample_rows=None)
        if hasattr(self.model, "graph_static_inputs"):
            fb.extra = self.model.graph_static_inputs(bs)
        if getattr(self.model, "lora_names", None):
            fb.lora_slots = torch.zeros(bs, dtype=torch.int32, device=d)
        if self.ep_group is not None:  # the bucket's exchange capacity is baked into its graph
            self.model.ep_capacity_tokens, self.model.ep_exact = bs, False
        s = torch.cuda.Stream(device=d)
        s.wait_stream(torch.cuda.current_stream(d))
        with torch.cuda.stream(s):
            for _ in range(2):
                self.model.forward(fb, self.kv, self.decode_ws)
        torch.cuda.current_stream(d).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with hip_graph_capture(g, s):
            logits = self.model.forward(fb, self.kv, self.decode_ws)
        self.graphs[bs] = (g, fb, logits)

    def capture_graphs(self, max_bs: Optional[int] = None):
        """Capture the decode graphs of every batch bucket <= max_bs. With TP, every rank calls this at the
        same point (the captures contain the collectives)."""
        if self.device.type != "cuda" or not (self.cfg.use_graphs or self.multi_graphs_ok):
            return
        for bs in self.cfg.graph_batch_sizes:
            if bs <= (max_bs or self.cfg.max_num_seqs):
                if self.cfg.use_graphs:
                    self._capture(bs)
                if self._multi_step_capable():
                    self._capture_multi(bs)

    # ------------------------------------------------------------------ multi-step decode
    def _multi_step_capable(self) -> bool:
        # EP lockstep steps one token at a time: every rank must enter the same number of exchanges per step
        return (self.cfg.decode_steps > 1 and self.ep_group is None and not hasattr(self.model, "graph_static_inputs")
                and not getattr(self.model, "lora_names", None))

    def _capture_multi(self, bs: int):
        K = self.cfg.decode_steps
        d = self.device
        ids = torch.zeros(bs, dtype=torch.int32, device=d)
        pos = torch.zeros(bs, dtype=torch.int32, device=d)
        slots = torch.full((bs,), self.pad_block * ops.BLOCK, dtype=torch.int32, device=d)
        ctx = torch.ones(bs, dtype=torch.int32, device=d)
        bt = torch.full((bs, self.max_blocks_per_seq), self.pad_block, dtype=torch.int32, device=d)
        samp = dict(temperature=torch.zeros(bs, dtype=torch.float32, device=d),
                    top_p=torch.ones(bs, dtype=torch.float32, device=d),
                    top_k=torch.zeros(bs, dtype=torch.int32, device=d),
                    seeds=torch.zeros(bs, dtype=torch.int64, device=d))
        n_valid = torch.zeros(1, dtype=torch.int32, device=d)
        toks = torch.zeros(K, bs, dtype=torch.int32, device=d)
        fb = ForwardBatch(token_ids=ids, positions=pos, slots=slots, num_prefill_tokens=0, decode_ctx=ctx,
                          decode_block_tables=bt, max_decode_ctx=self.cfg.max_model_len, sample_rows=None,
                          tp_local_logits=self.tp_size > 1 and getattr(self.model, "supports_tp_sampling", False))
        dctx = getattr(self.model, "ctx", None)
        # the closure holds the model / cache / workspace, never the engine: engine -> multi_graphs -> run -> engine
        # would be a reference cycle that keeps the whole engine (KV cache, graphs) alive after `del` until a GC pass
        model, kv, dws = self.model, self.kv, self.decode_ws

        def run():
            # every step first advances rows < n_valid from the previous sampled token: at j = 0 that is
            # toks[K-1], the last token of the previous run (pipelined) or the host-fed input token
            for j in range(K):
                ops.decode_advance(toks[(j - 1) % K], ids, pos, ctx, slots, bt, n_valid)
                logits = model.forward(fb, kv, dws)
                if fb.tp_local_logits:  # vocab-parallel logits: candidate exchange instead of a logits all-gather
                    ops.sample_tp(logits, dctx, model.vstart, model.cfg.vocab_size, samp["temperature"],
                                  samp["top_p"], samp["top_k"], samp["seeds"], j, out=toks[j])
                else:
                    ops.sample(logits, samp["temperature"], samp["top_p"], samp["top_k"], samp["seeds"], j,
                               out=toks[j])

        g = None
        if d.type == "cuda" and self.multi_graphs_ok:
            s = torch.cuda.Stream(device=d)
            s.wait_stream(torch.cuda.current_stream(d))
            with torch.cuda.stream(s):
                run()  # warm-up (n_valid = 0: the advance kernel touches no row)
            torch.cuda.current_stream(d).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with hip_graph_capture(g, s):
                run()
        self.multi_graphs[bs] = (g, run, fb, samp, n_valid, toks)

    def _worth_multi(self, reqs, extra: int = 0) -> bool:
        """A K-step run pays off when some row still needs >= 3K/4 tokens (rows that finish inside the run
        compute discarded tokens; a nearly-finished batch is cheaper as single steps). ``extra``: tokens
        per row already sampled by unprocessed runs."""
        K = self.cfg.decode_steps
        return max(r.max_new - len(r.output_ids) - extra for r in reqs) >= (3 * K) // 4

    def _multi_steps_for(self, b, reqs) -> int:
        """K if this pure-decode batch can run a K-step graph, else 1."""
        K = self.cfg.decode_steps
        if K <= 1 or not self._multi_step_capable() or self.sched.num_waiting() > 0:
            return 1
        if self._graph_bucket(len(reqs)) is None:
            return 1
        lim = self.cfg.max_model_len
        for r in reqs:
            if r is None or r.finished or r.params.has_penalty or r.params.guided is not None:
                return 1
            if len(r.prompt_ids) + len(r.output_ids) + K > lim:
                return 1
        return K if self._worth_multi(reqs) else 1

    def _run_seeds(self, reqs) -> np.ndarray:
        # per-run seed stream: the graph bakes the in-run step index, the host mixes in the engine step
        return (np.asarray([r.seed for r in reqs], np.int64) * np.int64(0x9E3779B1)
                + np.int64(self.step_count) * np.int64(0x632BE5AB)) & np.int64(0x7FFFFFFFFFFFFFFF)

    def _plan_multi(self, b, reqs, K: int) -> Optional[dict]:
        ids_list = list(b.decode_seq_ids)
        n = len(ids_list)
        bt_np = self.sched.reserve_decode(ids_list, K)
        if bt_np is None:
            return None
        params = [r.params for r in reqs]
        temp = np.fromiter((0.0 if p.top_k == 1 else p.temperature for p in params), np.float32, n)
        top_p = np.fromiter((p.top_p for p in params), np.float32, n)
        top_k = np.fromiter((p.top_k for p in params), np.int32, n)
        # host-fed first run: the graph's leading decode_advance moves (token, position - 1) to the input row
        return dict(op="multi", K=int(K), n=n, chained=False,
                    arr=[b.token_ids, np.asarray(b.positions, np.int32) - 1, bt_np, temp, top_p, top_k,
                         self._run_seeds(reqs), np.asarray([n], np.int32)])

    def _bank(self) -> HostStager:
        """Switch to the other staging bank for this launch (waits for that bank's previous copies)."""
        self._launches += 1
        self.stager = self.stagers[self._launches & 1]
        self.stager.reset()
        return self.stager

    def _exec_multi(self, plan: dict) -> Optional[tuple]:
        """Enqueue a K-step decode graph run from a plan (no host sync). The leader gets (host token
        buffer [K, bucket], completion event) back; followers None."""
        n, K = plan["n"], plan["K"]
        bs = self._graph_bucket(n)
        if bs not in self.multi_graphs:
            self._capture_multi(bs)
        g, run, fb, samp, n_valid, toks = self.multi_graphs[bs]
        st = self._bank()
        src = self._to_device(plan["arr"])
        if plan["chained"]:  # inputs are already on the device: new page tables and seeds only
            bt, seeds = src
            fb.decode_block_tables[:n, :bt.shape[1]].copy_(bt)
            samp["seeds"][:n].copy_(seeds)
        else:
            toks[K - 1, :n].copy_(src[0])
            fb.positions[:n].copy_(src[1])
            mb = plan["arr"][2].shape[1]
            fb.decode_block_tables[:n, :mb].copy_(src[2])
            if n < bs:
                fb.token_ids[n:].zero_()
                fb.positions[n:].zero_()
                fb.slots[n:].fill_(self.pad_block * ops.BLOCK)
                fb.decode_ctx[n:].fill_(1)
                fb.decode_block_tables[n:, 0].fill_(self.pad_block)
            samp["temperature"][:n].copy_(src[3])
            samp["top_p"][:n].copy_(src[4])
            samp["top_k"][:n].copy_(src[5])
            samp["seeds"][:n].copy_(src[6])
            n_valid.copy_(src[7])
        if g is not None:
            g.replay()
            self.stats["graph_steps"] += K
        else:
            run()  # eager (CPU / graphs off): same device-side feedback, no host round trip per token
        self.stats["multi_step_runs"] += 1
        out = None
        if self.leader:
            if self.device.type == "cuda":
                if self._tok_host is None:
                    cap = K * max(self.cfg.graph_batch_sizes)
                    self._tok_host = [torch.empty(cap, dtype=torch.int32, pin_memory=True) for _ in range(2)]
                buf = self._tok_host[self._launches & 1][:K * bs].view(K, bs)
                buf.copy_(toks, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                out = (buf.numpy(), ev)
            else:
                out = (toks.clone().numpy(), None)
        st.fence()
        self._step_done()
        return out

    def _launch_multi(self, b, reqs, K: int) -> Optional[_Run]:
        plan = self._plan_multi(b, reqs, K)
        if plan is None:
            return None
        self.step_count += K - 1
        self.stats["decode_tokens"] += plan["n"] * (K - 1)
        self._publish(plan)
        with roctx_range("decode_multi"):
            host, ev = self._exec_multi(plan)
        base = [int(p) for p in b.positions]
        return _Run([int(x) for x in b.decode_seq_ids], reqs, K, plan["n"], False, base, host, ev)

    def _chain(self, run: _Run) -> Optional[_Run]:
        """Enqueue run r+1 of a pending run r (before r's tokens are read), or None when the batch should
        go back to the scheduler: requests waiting, the bucket shrank, too few tokens left, no KV pages."""
        if not self._pipeline or self.sched.num_waiting() > 0:
            return None
        alive = [i for i, r in enumerate(run.reqs) if not r.finished]
        if not alive or self._graph_bucket(len(alive)) != self._graph_bucket(run.n):
            return None
        if self.sched.num_running() != len(alive):  # other running sequences must join the next batch
            return None
        K = run.K
        if not self._worth_multi([run.reqs[i] for i in alive], extra=K):
            return None
        base = [p + K for p in run.base]
        if max(base) + K > self.cfg.max_model_len:  # every row, finished ones included (page-table width)
            return None
        bt = self.sched.reserve_upto([run.ids[i] for i in alive], [base[i] + K for i in alive])
        if bt is None:
            return None
        full = np.full((run.n, bt.shape[1]), self.pad_block, np.int32)  # finished rows: scratch page
        full[alive] = bt
        self.step_count += K
        self.stats["steps"] += 1
        self.stats["chained_runs"] += 1
        self.stats["decode_tokens"] += len(alive) * K
        plan = dict(op="multi", K=K, n=run.n, chained=True,
                    arr=[full, self._run_seeds(run.reqs)])
        self._publish(plan)
        with roctx_range("decode_multi"):
            host, ev = self._exec_multi(plan)
        return _Run(run.ids, run.reqs, K, run.n, True, base, host, ev)

    def _complete(self, run: _Run) -> List[RequestOutput]:
        """Wait for a run's tokens and apply them (stop conditions, detokenisation, scheduler state)."""
        if run.done is not None:
            run.done.synchronize()
        self._mark("forward")
        host = run.host[:, :run.n]
        outs: List[RequestOutput] = []
        alive = [i for i in range(run.n) if not run.reqs[i].finished]
        for j in range(run.K):
            if not alive:
                break
            outs += self._process([run.ids[i] for i in alive], [run.reqs[i] for i in alive],
                                  host[j, alive].tolist(), defer_append=True)
            alive = [i for i in alive if not run.reqs[i].finished]
        if alive:
            self.sched.advance_decode([run.ids[i] for i in alive], host[:, alive].T.reshape(-1).tolist(), run.K,
                                      run.chained)
        self._mark("process")
        return outs

    def _plan_single(self, b) -> tuple:
        """(plan, seq_order) of a one-token step: a captured decode graph when the batch is pure decode and
        fits a bucket, otherwise an eager (prefill / mixed) forward. Sampling parameters ride along."""
        P, nd = b.num_prefill_tokens, len(b.decode_seq_ids)
        # EP lockstep: a pure-decode rank replays its graph only in a step every rank agreed to graph (_ep_bucket);
        # while a peer prefills, every rank runs eager with the exact-count exchange (the captured peer-memory
        # all-to-all would wait for a rank that is inside a different collective)
        ep_ok = self.ep_group is None or self._ep_bucket is not None
        if (P == 0 and ep_ok and self.device.type == "cuda" and self.cfg.use_graphs
                and self._graph_bucket(max(nd, self._ep_bucket or 0)) is not None):
            seq_order = [int(x) for x in b.decode_seq_ids]
            plan = dict(op="graph", n=nd, arr=[b.token_ids, b.positions, b.slots, b.decode_ctx,
                                                b.decode_block_tables], seq_ids=seq_order)
            if getattr(self.model, "lora_names", None):
                plan["lora"] = np.asarray([self._slot(s) for s in seq_order], np.int32)
        else:
            plan = self._plan_eager(b)
            seq_order = plan["pseq"] + [int(x) for x in b.decode_seq_ids]
        reqs = [self.requests.get(s) for s in seq_order]
        params = [r.params if r else SamplingParams() for r in reqs]
        plan["samp"] = SamplingBatch.arrays(params, [r.seed if r else 0 for r in reqs])
        plan["step"] = self.step_count
        return plan, seq_order, reqs

    def _exec_single(self, plan: dict, reqs=None, async_: bool = False):
        """Forward of a one-token step on this rank; the leader also samples (followers need no tokens:
        the next plan carries them). async_: return (pinned token buffer, completion event) instead of
        waiting for the tokens (GPU only)."""
        st = self._bank()
        if plan["op"] == "graph":
            logits = self._run_graph(plan)
        else:
            fb = self._batch_from_plan(plan)
            logits = self.model.forward(fb, self.kv, self.decode_ws)
            if fb.sample_rows.numel() == 0:
                logits = None
        self._mark("forward")
        toks = None
        if self.leader and logits is not None:
            self._penalize(logits, reqs)
            self._guide(logits, reqs)
            temp, top_p, top_k, seeds = self._to_device(plan["samp"])
            self._mark("penalize_pack")
            t = ops.sample(logits, temp, top_p, top_k, seeds, plan["step"])
            self._mark("sample")
            if async_ and self.device.type == "cuda" and not self._timing:
                n = t.shape[0]
                cap = max(self.cfg.max_num_seqs, max(self.cfg.graph_batch_sizes), n)
                if self._single_host is None or self._single_host[0].numel() < cap:
                    self._single_host = [torch.empty(cap, dtype=torch.int32, pin_memory=True) for _ in range(2)]
                buf = self._single_host[self._launches & 1][:n]
                buf.copy_(t, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                toks = (buf.numpy(), ev)
            else:
                toks = t.cpu().tolist()
        st.fence()
        self._step_done()
        return toks

    def _run_graph(self, plan: dict):
        n = plan["n"]
        bs = self._graph_bucket(max(n, self._ep_bucket or 0))
        if bs not in self.graphs:
            self._capture(bs)
        g, fb, logits = self.graphs[bs]
        arr = plan["arr"]
        src = self._to_device(arr)
        fb.token_ids[:n].copy_(src[0])
        fb.positions[:n].copy_(src[1])
        fb.slots[:n].copy_(src[2])
        fb.decode_ctx[:n].copy_(src[3])
        mb = arr[4].shape[1]
        fb.decode_block_tables[:n, :mb].copy_(src[4])
        if n < bs:  # padded rows: scratch page, ctx 1
            fb.slots[n:].fill_(self.pad_block * ops.BLOCK)
            fb.decode_ctx[n:].fill_(1)
            fb.decode_block_tables[n:, 0].fill_(self.pad_block)
        if fb.extra is not None:
            self.model.fill_graph_inputs(fb.extra, list(plan["seq_ids"]), n)
        if fb.lora_slots is not None:
            fb.lora_slots.zero_()
            fb.lora_slots[:n].copy_(self._to_device([plan["lora"]])[0])
        g.replay()
        self.stats["graph_steps"] += 1
        return logits[:n]

    # ------------------------------------------------------------------ step
    def _lookahead_ok(self) -> bool:
        """Schedule the next batch while a one-token step is in flight only when schedule() cannot preempt: a
        sequence whose token is still on the device must not be reset and re-admitted (its pending token would
        then be appended twice). Every running sequence needs at most one new KV page per step."""
        # only while prompts are still waiting for prefill: with none waiting the look-ahead batch would be the
        # decode of every running sequence EXCEPT the in-flight ones, splitting the decode batch in two (a
        # second, small-batch pass over all the decode steps)
        return (self._lookahead and self.ep_group is None and self.device.type == "cuda"
                and self.sched.num_waiting() > 0
                and self.sched.num_free_blocks() > self.sched.num_running() + 1)

    def _schedule_and_launch(self):
        """schedule() and enqueue the batch: a pending handle (_Run / _Single), None when nothing is scheduled
        or nothing was sampled, or a list of outputs (synchronous paths: EP lockstep, CPU)."""
        b = self.sched.schedule()
        self._mark("schedule")
        n_tok = b.num_tokens
        if self.ep_group is not None:
            t_max, any_prefill = self._ep_agree([n_tok, int(b.num_prefill_tokens > 0)])
            if t_max == 0:
                return None
            self.model.ep_capacity_tokens, self.model.ep_exact = t_max, bool(any_prefill)
            graphed = (not any_prefill and self.cfg.use_graphs and self.device.type == "cuda"
                       and self._graph_bucket(t_max) is not None)
            self._ep_bucket = t_max if graphed else None
            if n_tok == 0:
                if graphed:
                    self._ep_idle_graph(t_max)
                else:
                    self._ep_dummy_forward()
                return None
        if n_tok == 0:
            return None
        self.step_count += 1
        self.stats["steps"] += 1
        P = b.num_prefill_tokens
        self.stats["prefill_tokens"] += P
        self.stats["decode_tokens"] += n_tok - P
        nd = len(b.decode_seq_ids)
        if P == 0 and nd and self.cfg.decode_steps > 1:
            dreqs = [self.requests.get(s) for s in b.decode_seq_ids]
            K = self._multi_steps_for(b, dreqs)
            if K > 1:
                run = self._launch_multi(b, dreqs, K)
                if run is not None:
                    return run  # its tokens are processed by the next step(), after run 2 is enqueued
        plan, seq_order, reqs = self._plan_single(b)
        self._publish(plan)
        with roctx_range("prefill" if P else "decode"):
            toks = self._exec_single(plan, reqs, async_=self._lookahead and self.ep_group is None)
        if toks is None:
            return None
        if isinstance(toks, tuple):
            host, ev = toks
            return _Single(seq_order, reqs, len(seq_order), host, ev)
        out = self._process(seq_order, reqs, toks)
        self._mark("process")
        return out

    def _complete_single(self, p: _Single) -> List[RequestOutput]:
        if p.done is not None:
            p.done.synchronize()
        toks = p.host[:p.n].tolist() if hasattr(p.host, "tolist") else list(p.host)
        out = self._process(p.seq_order, p.reqs, toks)
        self._mark("process")
        return out

    @torch.inference_mode()
    def step(self) -> List[RequestOutput]:
        if not self.leader:
            raise RuntimeError("LLMEngine.step() runs on the TP leader; followers call follow()")
        with self.lock:
            if self._timing:
                self._t_mark = time.perf_counter()
            p = self._pending
            if isinstance(p, _Run):
                # pipelined decode: enqueue run r+1, then process run r while r+1 executes
                if self.host_timeline is not None:
                    t0 = time.perf_counter()
                    self._pending = self._chain(p)
                    t1 = time.perf_counter()
                    outs = self._complete(p)
                    self.host_timeline += [("chain" if self._pending is not None else "nochain", t0, t1),
                                           ("complete", t1, time.perf_counter())]
                    return outs
                self._pending = self._chain(p)
                return self._complete(p)
            if isinstance(p, _Single):
                # the next batch goes to the device before this step's tokens are read (its sequences are not
                # schedulable until they are: schedule() sees no uncomputed token for them)
                nxt = self._schedule_and_launch() if self._lookahead_ok() else None
                self._pending = None
                outs = self._complete_single(p)
                if isinstance(nxt, list):
                    return outs + nxt
                self._pending = nxt
                return outs
            nxt = self._schedule_and_launch()
            if isinstance(nxt, list):
                return nxt
            self._pending = nxt
            return []

    # ------------------------------------------------------------------ tensor-parallel followers
    @torch.inference_mode()
    def follow(self) -> str:
        """Follower ranks of a TP engine: execute rank 0's step plans until it yields ('yield': the caller's
        SPMD code continues, e.g. the next retrieval phase of a benchmark step) or stops ('stop')."""
        if self.leader or self.chan is None:
            raise RuntimeError("follow() runs on TP follower ranks")
        while True:
            plan = self.chan.recv()
            op = plan["op"]
            if op in ("yield", "stop"):
                return op
            if op == "multi":
                self._exec_multi(plan)
            elif op in ("graph", "eager"):
                self._exec_single(plan)
            elif op == "call" and plan["fn"] in self._REPLICATED:
                getattr(self, plan["fn"])(*plan["args"])
            else:
                raise RuntimeError(f"step channel: unknown plan op {op!r}")

    _REPLICATED = ("add_lora",)

    def release_followers(self, stop: bool = False) -> None:
        """Leader: hand control back to the followers' callers ('yield') or end their loops ('stop')."""
        if self.chan is not None and self.leader and not getattr(self, "_stopped", False):
            self.chan.send({"op": "stop" if stop else "yield"})
            self._stopped = stop

    def _mark(self, phase: str):
        """GAI_STEP_TIMING=1: synchronise and accumulate wall time per step phase in ``self.phase_ms``."""
        if not self._timing:
            return
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        self.phase_ms[phase] = self.phase_ms.get(phase, 0.0) + 1000 * (now - self._t_mark)
        self._t_mark = now

    def _penalize(self, logits, reqs):
        rows = [i for i, r in enumerate(reqs) if r is not None and r.params.has_penalty and r.token_counts]
        if not rows:
            return
        m = max(len(reqs[i].token_counts) for i in rows)
        ids = np.zeros((len(reqs), m), np.int32)
        cnt = np.zeros((len(reqs), m), np.int32)
        n = np.zeros(len(reqs), np.int32)
        f = np.zeros(len(reqs), np.float32)
        p = np.zeros(len(reqs), np.float32)
        rp = np.ones(len(reqs), np.float32)
        for i in rows:
            r = reqs[i]
            k = list(r.token_counts.items())
            ids[i, : len(k)] = [a for a, _ in k]
            cnt[i, : len(k)] = [c for _, c in k]
            n[i] = len(k)
            f[i], p[i], rp[i] = r.params.frequency_penalty, r.params.presence_penalty, r.params.repetition_penalty
        ops.apply_penalties(logits, *self.stager.stage([ids, cnt, n, f, p, rp]))

    def _guide(self, logits, reqs):
        """Constrained decoding: -inf on every token the grammar of a guided row does not allow next
        (host matcher masks -> token_mask HIP kernel), before sampling."""
        rows = [i for i, r in enumerate(reqs) if r is not None and r.matcher is not None and not r.finished]
        if not rows:
            return
        if self._masks is None:
            from .guided import MaskBuilder
            self._masks = MaskBuilder()
        words = (logits.shape[1] + 31) // 32
        gw = max(reqs[i].params.guided.words for i in rows)
        mask = self._masks.build(rows, [reqs[i].matcher for i in rows],
                                 [reqs[i].max_new - len(reqs[i].output_ids) for i in rows], gw)
        if gw < words:  # logits wider than the tokenizer's vocabulary: the extra ids stay disallowed
            mask = np.concatenate([mask, np.zeros((len(rows), words - gw), np.int32)], 1)
        mask = np.ascontiguousarray(mask[:, :words])
        for j, i in enumerate(rows):  # nothing allowed (budget exhausted): the request ends, its sample is dropped
            if not mask[j].any():
                reqs[i].mask_empty = True
                mask[j] = -1
        ops.token_mask(logits, *self._to_device([np.asarray(rows, np.int32), mask]))

    def _process(self, seq_order, reqs, toks, defer_append: bool = False) -> List[RequestOutput]:
        """Apply one sampled token per sequence. defer_append: the caller hands the tokens of
        continuing sequences to the scheduler itself (multi-step runs)."""
        outs: List[RequestOutput] = []
        cont_ids, cont_toks = [], []
        now = time.perf_counter()
        for sid, req, t in zip(seq_order, reqs, toks):
            if req is None or req.finished:
                continue
            if req.first_token_time is None:
                req.first_token_time = now
            if req.mask_empty:  # no token was allowed: finish without the (meaningless) sample
                req.finished, req.finish_reason, req.finish_time = True, "length", now
                self.sched.finish(sid)
                self.requests.pop(sid, None)
                self._release(sid)
                self.by_rid.pop(req.request_id, None)
                outs.append(RequestOutput(req.request_id, -1, req.detok.flush(), True, "length"))
                continue
            req.output_ids.append(t)
            if req.params.has_penalty:
                req.token_counts[t] = req.token_counts.get(t, 0) + 1
            if req.matcher is not None:
                req.matcher.advance(int(t))
            ntok = len(req.output_ids)
            reason = None
            is_eos = (t in self.eos and not req.params.ignore_eos) or t in req.params.stop_token_ids
            if is_eos and ntok > req.params.min_tokens:
                reason = "stop"
                delta = req.detok.flush()
            else:
                delta = req.detok.add(t)
                if req.detok.stopped:
                    reason = "stop"
                elif req.matcher is not None and (req.matcher.done or req.matcher.dead):
                    reason = "stop"  # the constrained value is complete
                elif ntok >= req.params.max_tokens or len(req.prompt_ids) + ntok >= self.cfg.max_model_len:
                    reason = "length"
                if reason:
                    delta += req.detok.flush()
            if reason:
                req.finished, req.finish_reason, req.finish_time = True, reason, now
                self.sched.finish(sid)
                self.requests.pop(sid, None)
                self._release(sid)
                self.by_rid.pop(req.request_id, None)
            else:
                cont_ids.append(sid)
                cont_toks.append(t)
            outs.append(RequestOutput(req.request_id, t, delta, reason is not None, reason))
        if cont_ids and not defer_append:
            self.sched.append_tokens(cont_ids, cont_toks)
        return outs

    # ------------------------------------------------------------------ offline API
    def generate(self, prompts: List[List[int]], params: SamplingParams | List[SamplingParams] | None = None
                 ) -> List[Request]:
        ps = params if isinstance(params, list) else [params or SamplingParams()] * len(prompts)
        reqs = [self.add_request(p, sp) for p, sp in zip(prompts, ps)]
        while self.has_work():
            self.step()
        return reqs

    # ------------------------------------------------------------------ teardown
    def close(self) -> None:
        """Release the engine's device state now: captured graphs (and their private memory pools), the paged KV
        cache, the decode workspace and the pinned staging banks. A replacement engine (hub reload, LoRA swap, a
        test) then sizes its KV cache against free memory, not against this engine's leftovers. The engine is
        unusable afterwards."""
        with self.lock:
            if self._pending is not None and self._pending.done is not None:
                self._pending.done.synchronize()
            self._pending = None
            self.graphs.clear()
            self.multi_graphs.clear()
            self.kv = None
            self.decode_ws = None
            self.stagers = []
            self.stager = None
            self._tok_host = self._single_host = None
            self.requests.clear()
            self.by_rid.clear()
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
                torch.cuda.empty_cache()
