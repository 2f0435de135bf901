"""FM-radio streaming RAG app (community/fm_asr; reference community/fm-asr-streaming-rag): the signal chain against
scipy.signal (the reference runs cupyx.scipy.signal with the same calls), the packet receiver, the speech-pipeline
plumbing, the transcript accumulator and its time-indexed database, intent-routed answers and the chain server."""
import zlib
import datetime as dt
import json
import math

import numpy as np
import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.community.fm_asr import dsp
from generativeaiexamples_amd.community.fm_asr.chains import StreamQuery, StreamRagChain, TimeResponse, first_json_object
from generativeaiexamples_amd.community.fm_asr.pipeline import (CallableAsr, PacketReceiver, SdrParams, SdrPipeline,
                                                               SignalChain)
from generativeaiexamples_amd.community.fm_asr.stream_store import (StreamRetriever, TextAccumulator,
                                                                   TimestampDatabase, drop_outliers)
from generativeaiexamples_amd.index.hbm_index import Document

signal = pytest.importorskip("scipy.signal")


def _fm_burst(n=20000, fs=1e6, tone=1000.0, dev=75e3, seed=0):
    """An FM-modulated tone plus noise, complex64 baseband."""
    t = np.arange(n) / fs
    msg = np.sin(2 * np.pi * tone * t)
    phase = 2 * np.pi * dev * np.cumsum(msg) / fs
    rng = np.random.default_rng(seed)
    x = np.exp(1j * phase) + 0.05 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    return x.astype(np.complex64)


def test_firwin_matches_scipy():
    for n, fc, fs in ((101, 100e3, 1e6), (31, 0.25, 2.0), (2501, 1 / 125, 2.0)):
        np.testing.assert_allclose(dsp.firwin(n, fc, fs=fs), signal.firwin(n, fc, window="hamming", fs=fs),
                                   rtol=1e-9, atol=1e-12)


def test_lowpass_demod_resample_match_scipy():
    x = _fm_burst()
    taps = dsp.firwin(101, 100e3, fs=1e6)
    y = dsp.lowpass(taps, torch.from_numpy(x)).numpy()
    ref = signal.lfilter(taps, [1.0], x)
    np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-5)
    d = dsp.fm_demod(torch.from_numpy(y)).numpy()
    dref = np.diff(np.unwrap(np.angle(ref)))
    np.testing.assert_allclose(d, dref, atol=2e-4)
    for up, down in ((2, 125), (1, 62), (3, 2)):
        r = dsp.resample_poly(torch.from_numpy(d), up, down).numpy()
        rref = signal.resample_poly(d, up, down, window="hamming")
        assert r.shape == rref.shape
        np.testing.assert_allclose(r, rref, rtol=1e-4, atol=1e-5)
    assert dsp.rational_factors(1e6, 16e3) == (2, 125)


def test_signal_chain_recovers_tone_and_pcm():
    p = SdrParams()
    chain = SignalChain(p, device="cpu")
    audio = chain(torch.from_numpy(_fm_burst(n=62500)))
    assert audio.numel() == math.ceil((62500 - 1) * 2 / 125)  # one fewer sample after the discriminator
    spec = np.abs(np.fft.rfft(audio.numpy()[50:] * np.hanning(audio.numel() - 50)))
    f = np.fft.rfftfreq(audio.numel() - 50, 1 / 16000.0)
    assert abs(f[spec.argmax()] - 1000.0) < 40.0  # the modulating tone comes back
    pcm = dsp.float_to_pcm16(torch.tensor([0.0, 0.5, -1.5, 2.0]))
    assert pcm.tolist() == [0, 16384, -32768, 32767]


def test_packet_receiver_bursts_and_params(tmp_path):
    p = SdrParams(batch_size=64, header_bytes=8)
    rx = PacketReceiver(p)
    samples = np.arange(20, dtype=np.float32).view(np.complex64)  # 10 complex samples = 80 B
    bursts = []
    for i in range(0, 80, 16):
        b = rx.feed(b"HEADER!!" + samples.tobytes()[i:i + 16])
        if b is not None:
            bursts.append(b)
    assert len(bursts) == 1 and bursts[0].dtype == np.complex64 and len(bursts[0]) == 8  # 64 payload bytes
    np.testing.assert_array_equal(bursts[0], samples[:8])
    assert len(rx.burst.data) == 16 and bytes(rx.burst.header) == b"HEADER!!"  # the next burst has begun
    yml = tmp_path / "params.yml"
    yml.write_text("sensor:\n  sample_rate: 2000000\nnetwork_rx:\n  dst_port: 6000\nresample:\n  gain: 4.0\n")
    q = SdrParams.from_yaml(str(yml))
    assert (q.sample_rate, q.dst_port, q.gain, q.numtaps) == (2000000, 6000, 4.0, 101)


def test_pipeline_feeds_recogniser_in_one_second_pieces():
    got, texts = [], []
    asr = CallableAsr(lambda pcm: (got.append(len(pcm)), f"piece {len(got)}")[1])
    # 5 bursts of 62,500 samples (62.5 ms each at 1 MS/s) -> 5 x 1,000 audio samples = 10,000 PCM bytes, handed to
    # the recogniser in 4,000-byte pieces (the default piece is one second, 32,000 bytes) plus the flushed rest
    pipe = SdrPipeline(SdrParams(pcm_chunk_bytes=4000), asr, texts.append, device="cpu")
    for s in range(5):
        pipe.process_burst(_fm_burst(n=62500, seed=s))
    pipe.close()
    assert got == [4000, 4000, 2000]  # ceil(62,499 x 2 / 125) = 1,000 audio samples per burst
    assert texts == ["piece 1", "piece 2", "piece 3"] and pipe.errors == 0


def test_timestamp_db_and_accumulator():
    now = [dt.datetime(2024, 1, 1, 12, 0, 0)]
    db = TimestampDatabase(clock=lambda: now[0])
    acc = TextAccumulator(None, chunk_size=40, chunk_overlap=0, timestamp_db=db)
    r = acc.update("s1", "alpha beta gamma delta")
    assert r == {"status": "Added 0 entries"} and acc.pending("s1") == "alpha beta gamma delta"
    now[0] += dt.timedelta(minutes=5)
    r = acc.update("s1", "epsilon zeta eta theta iota kappa lambda mu")
    assert r["status"].startswith("Added") and len(db) >= 1
    assert acc.pending("s1") and acc.pending("s2") == ""
    assert len(db.recent(now[0] - dt.timedelta(minutes=1))) == len(db)
    assert db.recent(now[0] + dt.timedelta(seconds=1)) == []
    assert len(db.past(now[0] - dt.timedelta(minutes=4), window=90)) == 0
    assert len(db.past(now[0] - dt.timedelta(seconds=30), window=90)) == len(db)


class _HashEmb(Embeddings):
    dim = 64

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().split():
                out[i, zlib.crc32(w.strip(".,?").encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


class _ScriptedLLM:
    """Answers the intent / time prompts from a script and echoes the RAG context."""

    def __init__(self, intent, time_reply='{"timeNum": 10, "timeUnit": "minutes"}'):
        self.intent, self.time_reply, self.calls = intent, time_reply, []

    def invoke(self, messages, **kw):
        sys_ = messages[0]["content"]
        self.calls.append(sys_[:20])
        if "sort questions" in sys_:
            return f'Sure! {{"intentType": "{self.intent}"}}'
        if "amount of time" in sys_:
            return self.time_reply
        return "summary of " + messages[1]["content"][:30]

    def stream(self, messages, **kw):
        yield "ANSWER<" + messages[-1]["content"] + ">"


def _setup(clock):
    store = VectorStore("fm", _HashEmb(), device="cpu")
    ret = StreamRetriever(store)
    db = TimestampDatabase(clock=clock)
    acc = TextAccumulator(ret, chunk_size=60, chunk_overlap=0, timestamp_db=db)
    return acc, ret


def test_chain_routes_by_intent():
    now = [dt.datetime(2024, 1, 1, 12, 0, 0)]
    clock = lambda: now[0]  # noqa: E731
    acc, ret = _setup(clock)
    for i, topic in enumerate(["weather storm warning tonight", "football match results", "traffic jam highway"]):
        acc.update("radio", (topic + " ") * 8)
        now[0] += dt.timedelta(minutes=20)
    acc.update("radio", "closing words " * 10)
    # similarity
    out = "".join(StreamRagChain(_ScriptedLLM("SpecificTopic"), acc, ret, clock).answer(
        StreamQuery("any football results?", max_docs=2)))
    assert out.startswith("*Returned") and "football" in out
    # recent summary: only chunks stored in the last 10 minutes
    out = "".join(StreamRagChain(_ScriptedLLM("RecentSummary"), acc, ret, clock).answer(
        StreamQuery("what was said in the last ten minutes?")))
    # (a chunk is stamped when it is finalized: the pending tail of the traffic report went in with the closing words)
    ctx = out.split("ANSWER<")[-1]
    assert "entries from the last 600s" in out and "closing" in ctx and "weather" not in ctx and "football" not in ctx
    # time window: around 40 minutes ago
    llm = _ScriptedLLM("TimeWindow", '{"timeNum": 40, "timeUnit": "min"}')
    out = "".join(StreamRagChain(llm, acc, ret, clock).answer(StreamQuery("what was on 40 minutes ago?")))
    assert "from 2400s ago" in out and "football" in out
    # unparseable time -> falls back to similarity
    llm = _ScriptedLLM("RecentSummary", "no idea")
    out = "".join(StreamRagChain(llm, acc, ret, clock).answer(StreamQuery("recap please")))
    assert out.startswith("*Returned") or out.startswith("*Found no")
    # summarization path when too many chunks
    out = "".join(StreamRagChain(_ScriptedLLM("RecentSummary", '{"timeNum": 2, "timeUnit": "hours"}'), acc, ret,
                                 clock).answer(StreamQuery("recap the last two hours", max_docs=1, allow_summary=True)))
    assert "Using summarization" in out
    # no knowledge base: plain chat
    out = "".join(StreamRagChain(_ScriptedLLM("Unknown"), acc, ret, clock).answer(
        StreamQuery("hello", use_knowledge_base=False)))
    assert out == "ANSWER<hello>"


def test_helpers():
    assert first_json_object("x {bad} y {'intentType': 'TimeWindow'}") == {"intentType": "TimeWindow"}
    assert TimeResponse(1.5, "Hours").to_seconds() == 5400 and TimeResponse(3, "sec").to_seconds() == 3
    with pytest.raises(ValueError):
        TimeResponse(1, "fortnights").to_seconds()
    docs = [Document(str(s), {"relevance_score": s}) for s in (10.0, 9.5, 9.0, 2.0, 1.0, 0.5)]
    assert [d.page_content for d in drop_outliers(docs)] == ["10.0", "9.5", "9.0"]


def test_chain_server_endpoints():
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.community.fm_asr.server import create_app

    acc, ret = _setup(dt.datetime.now)
    app = create_app(lambda: _ScriptedLLM("SpecificTopic"), acc, ret, lambda: ["meta/llama3-8b-instruct"])
    c = TestClient(app)
    assert c.get("/serverStatus").json() == {"is_ready": True}
    assert c.get("/availableNvidiaModels").json()["local_models"] == ["meta/llama3-8b-instruct"]
    for _ in range(6):
        r = c.post("/storeStreamingText", json={"transcript": "the mayor opened the new bridge today", "source_id": "k1"})
        assert r.status_code == 200 and r.json()["status"].startswith("Added")
    r = c.request("GET", "/generate", content=json.dumps({"question": "what did the mayor open?", "max_docs": 3}))
    assert r.status_code == 200 and "bridge" in r.text
    r = c.post("/generate", json={"question": "hi", "use_knowledge_base": False})
    assert r.text == "ANSWER<hi>"
    assert c.post("/generate", json={"max_docs": 3}).status_code == 422
    assert c.request("GET", "/generate", content=json.dumps({"max_docs": 3})).status_code == 422
