"""Failure detection / fault injection on the CPU tier: a rank killed mid-run is
detected as RankFailure by its peer (no hang), injected collective delays are observed, and the
serving engine's watchdog fails requests of a hung step and reports unhealthy."""
import asyncio
import socket
import time

import pytest
import torch.multiprocessing as mp

from tests import _dist_workers as W


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(180)
def test_killed_rank_is_detected(tmp_path):
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=W.fault_worker, args=(r, 2, port, str(tmp_path), "kill")) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert procs[1].exitcode == 17  # injected crash
    status = (tmp_path / "fault_kill_0.txt").read_text().splitlines()
    assert status[0].startswith("rank_failure"), status
    assert "tp_all_reduce" in status[0]


@pytest.mark.timeout(180)
def test_injected_delay(tmp_path):
    mp.spawn(W.fault_worker, args=(2, _port(), str(tmp_path), "delay"), nprocs=2, join=True)
    s0 = (tmp_path / "fault_delay_0.txt").read_text().splitlines()
    assert s0[0] == "ok" and float(s0[1]) > 6 * 0.3 * 0.9  # rank 0 waited for the delayed peer
    assert float(s0[2]) == 2.0 ** 6


def test_watchdog_fails_hung_step():
    from generativeaiexamples_amd.engine.llm_engine import RequestOutput
    from generativeaiexamples_amd.serving.async_engine import AsyncLLMEngine

    class Req:
        finished = False

    class HungEngine:
        tok = None

        def __init__(self):
            self.work = False

        def add_request(self, ids, params, rid, images=None, lora=None):
            self.work = True
            return Req()

        def has_work(self):
            return self.work

        def step(self):
            time.sleep(3.0)
            return [RequestOutput("x", 1, "a", True, "stop")]

        def abort(self, rid):
            return True

    eng = AsyncLLMEngine(HungEngine(), watchdog_s=0.5)

    async def go():
        out = []
        with pytest.raises(RuntimeError, match="watchdog"):
            async for it in eng.generate([1, 2, 3], None, "r1"):
                out.append(it)

    t0 = time.perf_counter()
    asyncio.run(go())
    assert time.perf_counter() - t0 < 2.5  # failed by the watchdog, not after the 3 s step
    assert not eng.healthy
    eng.shutdown()


class _SlowEngine:
    """Fake engine: every step takes 0.3 s and emits one finishing token for each admitted request."""
    tok = None

    def __init__(self, step_s=0.3):
        self.step_s, self.live, self.admitted = step_s, [], []
        self.stats = dict(prefill_tokens=0, decode_tokens=0)

    def add_request(self, ids, params, rid, images=None, lora=None):
        self.admitted.append(rid)
        self.live.append(rid)

        class Req:
            finished = False
            output_ids = [1]
            first_token_time = None
        return Req()

    def has_work(self):
        return bool(self.live)

    def step(self):
        from generativeaiexamples_amd.engine.llm_engine import RequestOutput
        time.sleep(self.step_s)
        outs = [RequestOutput(r, 7, "a", True, "stop") for r in self.live]
        self.live = []
        return outs

    def abort(self, rid):
        return True


def test_cancel_during_admission_keeps_engine_alive():
    """a client that disconnects while its admission waits in the inbox must be skipped, and the
    engine thread must keep serving later requests."""
    from generativeaiexamples_amd.serving.async_engine import AsyncLLMEngine
    fake = _SlowEngine()
    eng = AsyncLLMEngine(fake, watchdog_s=30)

    async def consume(rid):
        return [it async for it in eng.generate([1, 2], None, rid)]

    async def go():
        busy = asyncio.create_task(consume("busy"))  # keeps the engine thread inside a 0.3 s step
        await asyncio.sleep(0.1)
        victim = asyncio.create_task(consume("victim"))  # its admission now waits in the inbox
        await asyncio.sleep(0.05)
        victim.cancel()
        with pytest.raises(asyncio.CancelledError):
            await victim
        assert len(await busy) == 1
        after = await asyncio.wait_for(consume("after"), timeout=5)
        assert len(after) == 1 and after[0].finished

    asyncio.run(go())
    assert eng.thread.is_alive() and eng.healthy
    assert "victim" not in fake.admitted  # cancelled before it ran: never half-applied
    eng.shutdown()


def test_watchdog_fails_new_admissions_fast():
    """while a step is hung, new requests fail with the engine error instead of waiting."""
    from generativeaiexamples_amd.serving.async_engine import AsyncLLMEngine
    eng = AsyncLLMEngine(_SlowEngine(step_s=3.0), watchdog_s=0.4)

    async def go():
        first = asyncio.create_task(eng.complete([1], None, "r0"))
        await asyncio.sleep(1.0)  # the watchdog has fired on the hung step
        t0 = time.perf_counter()
        with pytest.raises(TimeoutError):
            await eng.complete([1], None, "r1")
        assert time.perf_counter() - t0 < 0.5
        with pytest.raises(RuntimeError):
            await first

    asyncio.run(go())
    assert not eng.healthy
    eng.shutdown()


def test_ep_exchange_error_word_raises_and_retires(tmp_path):
    """an expert-parallel engine polls its peer-memory all-to-all's error word at the end of
    every step; a set word raises RankFailure and retires the exchange (no stale-slot tokens are returned)."""
    import torch
    import torch.distributed as dist

    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models.mixtral import MixtralConfig, MixtralModel
    from generativeaiexamples_amd.parallel.custom_ar import CustomAllReduce
    from generativeaiexamples_amd.parallel.dist import DistContext
    from generativeaiexamples_amd.parallel.fault import RankFailure

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        m = MixtralModel(MixtralConfig.tiny_moe(), device="cpu", dtype=torch.float32, dist_ctx=DistContext(),
                         ep_group=dist.group.WORLD).random_init(1)

        class FakeXchg:  # the error word of a CustomAllReduce after a peer missed the bounded spin
            err = torch.ones(1, dtype=torch.int32)
            rank = 0
            check = CustomAllReduce.check

            def eligible_a2a(self, t):  # no peer buffers: the exchange itself takes the gloo path
                return False

        m.ep_xchg = FakeXchg()
        eng = LLMEngine(m, small_byte_tokenizer(512), EngineConfig(num_blocks=32, max_model_len=64, use_graphs=False))
        eng.add_request([5, 6, 7], SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True))
        with pytest.raises(RankFailure):
            while eng.has_work():
                eng.step()
        assert m.ep_xchg is None
        FakeXchg.err.zero_()
    finally:
        dist.destroy_process_group()
