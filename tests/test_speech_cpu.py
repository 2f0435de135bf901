"""Speech playground (U7): the Riva-method gRPC client (descriptor-built messages) against an in-process
fake Riva server, and the playground's /speech routes. Wire compatibility with a real Riva server is
unverified offline (parity unpinned): this pins the client's protocol behaviour - config-first request
stream, finals + current partial transcript, 300-character TTS segmentation."""
import io
import json
import wave
from concurrent import futures

import grpc
import pytest

from generativeaiexamples_amd.playground import speech as S


class FakeRiva:
    """Echo ASR: reports the audio length it has seen as interim then final results; TTS: one chunk of
    int16 silence per request whose length encodes the request's text length."""

    def __init__(self):
        self.asr_configs, self.tts_texts = [], []

    def asr(self, req_iter, ctx):
        first = next(req_iter)
        self.asr_configs.append(first.streaming_config)
        total = 0
        for r in req_iter:
            total += len(r.audio_content)
            res = S.MSG["StreamingRecognitionResult"](is_final=False)
            res.alternatives.add(transcript=f"partial{total}")
            yield S.MSG["StreamingRecognizeResponse"](results=[res])
            if total >= 3200 * 2:  # a final every ~0.2 s of 16 kHz audio
                fin = S.MSG["StreamingRecognitionResult"](is_final=True)
                fin.alternatives.add(transcript=f"[{total}] ")
                yield S.MSG["StreamingRecognizeResponse"](results=[fin])
                total = 0

    def tts(self, req, ctx):
        self.tts_texts.append((req.text, req.voice_name, req.sample_rate_hz))
        yield S.MSG["SynthesizeSpeechResponse"](audio=b"\x00\x00" * len(req.text))


@pytest.fixture
def riva():
    fake = FakeRiva()
    srv = grpc.server(futures.ThreadPoolExecutor(4))
    handlers = {
        "StreamingRecognize": grpc.stream_stream_rpc_method_handler(
            fake.asr, request_deserializer=S.MSG["StreamingRecognizeRequest"].FromString,
            response_serializer=lambda m: m.SerializeToString()),
    }
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("nvidia.riva.asr.RivaSpeechRecognition", handlers),
                                  grpc.method_handlers_generic_handler("nvidia.riva.tts.RivaSpeechSynthesis", {
                                      "SynthesizeOnline": grpc.unary_stream_rpc_method_handler(
                                          fake.tts, request_deserializer=S.MSG["SynthesizeSpeechRequest"].FromString,
                                          response_serializer=lambda m: m.SerializeToString())})))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    yield fake, S.RivaBackend(f"127.0.0.1:{port}")
    srv.stop(0)


def test_asr_stream_and_transcript_assembly(riva):
    fake, be = riva
    pcm = S.tone(440, 0.5, 16000)  # 16000 B
    outs = list(be.transcribe(S.pcm_chunks(pcm, 16000, ms=100), "en-US", 16000))
    cfg = fake.asr_configs[0]
    assert cfg.config.sample_rate_hertz == 16000 and cfg.config.language_code == "en-US" and cfg.interim_results
    assert cfg.config.encoding == S.LINEAR_PCM and cfg.config.enable_automatic_punctuation
    assert outs[-1].startswith("[6400] [6400] ")  # two finals, then the running partial
    assert all(o.startswith(outs[i - 1].split("partial")[0]) for i, o in enumerate(outs) if i)


def test_tts_segments_long_text(riva):
    fake, be = riva
    text = " ".join(f"word{i}" for i in range(150))  # ~1000 characters
    pcm = b"".join(be.synthesize(text, "en-US", "English-US.Female-1"))
    assert len(fake.tts_texts) == 4 and all(len(t) <= 300 for t, _, _ in fake.tts_texts)
    assert " ".join(t for t, _, _ in fake.tts_texts) == text
    assert fake.tts_texts[0][1] == "English-US.Female-1" and fake.tts_texts[0][2] == be.sample_rate_tts
    assert len(pcm) == 2 * sum(len(t) for t, _, _ in fake.tts_texts)


def test_wav_roundtrip_and_resampling():
    pcm = S.tone(300, 0.25, 48000)
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(48000)
        import numpy as np

        x = np.frombuffer(pcm, np.int16)
        w.writeframes(np.stack([x, x], 1).tobytes())
    out = S.wav_to_pcm16(buf.getvalue(), 16000)
    assert abs(len(out) // 2 - 4000) <= 1
    wv = S.pcm_to_wav(out, 16000)
    with wave.open(io.BytesIO(wv)) as w:
        assert w.getframerate() == 16000 and w.getnchannels() == 1


def test_playground_speech_routes(riva):
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.playground.app import create_app

    fake, be = riva

    class NoChain:
        def health(self):
            return "down"

    c = TestClient(create_app("http://x", "m", client=NoChain(), speech=be))
    assert c.get("/api/speech/status").json()["asr"] is True
    assert b"Record" in c.get("/speech").content
    r = c.post("/api/speech/asr?language=en-US", content=S.pcm_to_wav(S.tone(440, 0.3, 16000), 16000))
    assert r.status_code == 200 and "[6400]" in r.json()["transcript"]
    r = c.post("/api/speech/tts", json={"text": "hello from the MI355X", "voice": "v"})
    assert r.status_code == 200 and r.headers["content-type"] == "audio/wav"
    off = TestClient(create_app("http://x", "m", client=NoChain(), speech=S.SpeechBackend()))
    assert off.get("/api/speech/status").json()["asr"] is False
    assert off.post("/api/speech/tts", json={"text": "x"}).status_code == 503


def test_asr_messages_match_reference_proto():
    """Pin the hand-built Riva ASR messages against the reference's riva_asr.proto (field numbers by name):
    every ASR field this client sends or reads must carry the proto's number."""
    import os
    import re

    import pytest

    from generativeaiexamples_amd.playground.speech import MSG

    path = ("/root/reference/community/pdfspeak/webapp/src/main/ui/web/pdf-speak/server/modules/protos/src/"
            "riva_proto/riva_asr.proto")
    if not os.path.exists(path):
        pytest.skip("reference proto not available")
    src = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    fields = {}
    for m in re.finditer(r"\bmessage\s+(\w+)\s*\{", src):
        depth, i = 1, m.end()
        while depth and i < len(src):
            depth += {"{": 1, "}": -1}.get(src[i], 0)
            i += 1
        body = src[m.end():i - 1]
        body = re.sub(r"\bmessage\s+\w+\s*\{.*?\}", "", body, flags=re.S)  # nested messages are their own entries
        fields[m.group(1)] = {f: int(n) for f, n in re.findall(r"(\w+)\s*=\s*(\d+)\s*;", body)}
    asr = ["RecognitionConfig", "StreamingRecognitionConfig", "StreamingRecognizeRequest",
           "SpeechRecognitionAlternative", "StreamingRecognitionResult", "StreamingRecognizeResponse"]
    checked = 0
    for name in asr:
        assert name in fields, name
        for f in MSG[name].DESCRIPTOR.fields:
            assert f.name in fields[name], (name, f.name)
            assert fields[name][f.name] == f.number, (name, f.name, f.number, fields[name][f.name])
            checked += 1
    assert checked >= 15
