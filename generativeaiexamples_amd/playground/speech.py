"""Speech for the playground (U7): streaming ASR for the question box and TTS for the answer.

The reference's speech playground (RAG/src/rag_playground/speech/asr_utils.py:117-170, tts_utils.py:83-135)
talks to a Riva server through the ``riva.client`` package; that package and its generated protobuf
modules are not installable offline, so this module speaks the same gRPC methods with message classes
built at import time from descriptors (google.protobuf, grpcio):

* ``/nvidia.riva.asr.RivaSpeechRecognition/StreamingRecognize`` - bidi stream: a first request with the
  StreamingRecognitionConfig (LINEAR_PCM, 16 kHz mono, language, automatic punctuation, interim results),
  then raw 16-bit PCM chunks; responses carry partial / final transcripts (the reference concatenates
  finals + the current partial, print_streaming_response);
* ``/nvidia.riva.tts.RivaSpeechSynthesis/SynthesizeOnline`` - server stream of int16 PCM chunks; long
  answers are split at ~300 characters on word boundaries (the reference's 400-character Riva limit).

The ASR messages are pinned field by field against the reference's riva_asr.proto
(community/pdfspeak/.../riva_proto/riva_asr.proto, tests/test_speech_cpu.py); the reference ships no TTS
proto, so the TTS field numbers remain parity-unpinned. The client / test server pair in
tests/test_speech_cpu.py pins the behaviour. The backend is pluggable (:class:`SpeechBackend`): ``RIVA_API_URI`` selects
:class:`RivaBackend`; without it the speech routes report that speech is unavailable, as the reference
does when no Riva server answers.
"""
from __future__ import annotations

import io
import os
import struct
import wave
from typing import Dict, Iterable, Iterator, List, Optional

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

# ------------------------------------------------------------------------------------------ messages
_F = descriptor_pb2.FieldDescriptorProto


def _field(msg, name, num, typ, label=_F.LABEL_OPTIONAL, type_name=None, oneof=None):
    f = msg.field.add(name=name, number=num, type=typ, label=label)
    if type_name:
        f.type_name = type_name
    if oneof is not None:
        f.oneof_index = oneof
    return f


def _build_messages():
    fd = descriptor_pb2.FileDescriptorProto(name="gai_riva_speech.proto", package="nvidia.riva", syntax="proto3")
    rc = fd.message_type.add(name="RecognitionConfig")
    _field(rc, "encoding", 1, _F.TYPE_INT32)  # AudioEncoding enum: 1 = LINEAR_PCM
    _field(rc, "sample_rate_hertz", 2, _F.TYPE_INT32)
    _field(rc, "language_code", 3, _F.TYPE_STRING)
    _field(rc, "max_alternatives", 4, _F.TYPE_INT32)
    _field(rc, "audio_channel_count", 7, _F.TYPE_INT32)
    _field(rc, "enable_automatic_punctuation", 11, _F.TYPE_BOOL)
    _field(rc, "model", 13, _F.TYPE_STRING)
    src = fd.message_type.add(name="StreamingRecognitionConfig")
    _field(src, "config", 1, _F.TYPE_MESSAGE, type_name=".nvidia.riva.RecognitionConfig")
    _field(src, "interim_results", 2, _F.TYPE_BOOL)
    req = fd.message_type.add(name="StreamingRecognizeRequest")
    req.oneof_decl.add(name="streaming_request")
    _field(req, "streaming_config", 1, _F.TYPE_MESSAGE, type_name=".nvidia.riva.StreamingRecognitionConfig", oneof=0)
    _field(req, "audio_content", 2, _F.TYPE_BYTES, oneof=0)
    alt = fd.message_type.add(name="SpeechRecognitionAlternative")
    _field(alt, "transcript", 1, _F.TYPE_STRING)
    _field(alt, "confidence", 2, _F.TYPE_FLOAT)
    res = fd.message_type.add(name="StreamingRecognitionResult")
    _field(res, "alternatives", 1, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, ".nvidia.riva.SpeechRecognitionAlternative")
    _field(res, "is_final", 2, _F.TYPE_BOOL)
    _field(res, "stability", 3, _F.TYPE_FLOAT)
    rsp = fd.message_type.add(name="StreamingRecognizeResponse")
    _field(rsp, "results", 1, _F.TYPE_MESSAGE, _F.LABEL_REPEATED, ".nvidia.riva.StreamingRecognitionResult")
    tts = fd.message_type.add(name="SynthesizeSpeechRequest")
    _field(tts, "text", 1, _F.TYPE_STRING)
    _field(tts, "language_code", 2, _F.TYPE_STRING)
    _field(tts, "encoding", 3, _F.TYPE_INT32)
    _field(tts, "sample_rate_hz", 4, _F.TYPE_INT32)
    _field(tts, "voice_name", 5, _F.TYPE_STRING)
    tr = fd.message_type.add(name="SynthesizeSpeechResponse")
    _field(tr, "audio", 1, _F.TYPE_BYTES)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return {m.name: get(pool.FindMessageTypeByName("nvidia.riva." + m.name)) for m in fd.message_type}


MSG = _build_messages()
ASR_METHOD = "/nvidia.riva.asr.RivaSpeechRecognition/StreamingRecognize"
TTS_METHOD = "/nvidia.riva.tts.RivaSpeechSynthesis/SynthesizeOnline"
LINEAR_PCM = 1


def split_for_tts(text: str, limit: int = 300) -> List[str]:
    """Pieces of at most ~limit characters, cut on word boundaries (tts_utils.text_to_speech)."""
    out, cur = [], ""
    for w in text.split():
        if cur and len(cur) + 1 + len(w) > limit:
            out.append(cur)
            cur = w
        else:
            cur = f"{cur} {w}" if cur else w
    if cur:
        out.append(cur)
    return out


def pcm_to_wav(pcm: bytes, rate: int) -> bytes:
    buf = io.BytesIO()
    with wave.open(buf, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(pcm)
    return buf.getvalue()


def wav_to_pcm16(data: bytes, rate: int = 16000) -> bytes:
    """A WAV upload (any channel count, 8/16-bit) -> mono int16 PCM at `rate` (linear resampling)."""
    import numpy as np

    with wave.open(io.BytesIO(data), "rb") as w:
        ch, sw, sr, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if sw == 2:
        x = np.frombuffer(raw, np.int16).astype(np.float32)
    elif sw == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) * 256.0
    else:
        raise ValueError(f"unsupported sample width {sw}")
    if ch > 1:
        x = x.reshape(-1, ch).mean(1)  # the reference averages channels too
    if sr != rate and len(x):
        t = np.arange(0, len(x) * rate / sr) * (sr / rate)
        x = np.interp(t, np.arange(len(x)), x)
    return np.clip(x, -32768, 32767).astype(np.int16).tobytes()


# ------------------------------------------------------------------------------------------ backends
class SpeechBackend:
    sample_rate_tts = 48000

    def available(self) -> bool:
        return False

    def transcribe(self, pcm_chunks: Iterable[bytes], language: str = "en-US", rate: int = 16000) -> Iterator[str]:
        """Yields the running transcript (finals so far + current partial)."""
        raise NotImplementedError

    def synthesize(self, text: str, language: str = "en-US", voice: str = "") -> Iterator[bytes]:
        """Yields int16 PCM chunks at ``sample_rate_tts``."""
        raise NotImplementedError


class RivaBackend(SpeechBackend):
    def __init__(self, uri: str, use_ssl: bool = False, api_key: Optional[str] = None,
                 function_ids: Optional[Dict[str, str]] = None):
        import grpc

        self.sample_rate_tts = int(os.environ.get("TTS_SAMPLE_RATE", 48000))
        creds = grpc.ssl_channel_credentials() if use_ssl else None
        self.channel = grpc.secure_channel(uri, creds) if creds else grpc.insecure_channel(uri)
        self.meta = []
        if api_key:  # hosted Riva (NVCF): bearer key + per-service function id
            self.meta.append(("authorization", f"Bearer {api_key}"))
        self.function_ids = function_ids or {}
        ser = lambda m: m.SerializeToString()  # noqa: E731
        self._asr = self.channel.stream_stream(ASR_METHOD, request_serializer=ser,
                                               response_deserializer=MSG["StreamingRecognizeResponse"].FromString)
        self._tts = self.channel.unary_stream(TTS_METHOD, request_serializer=ser,
                                              response_deserializer=MSG["SynthesizeSpeechResponse"].FromString)

    def available(self) -> bool:
        return True

    def _md(self, service: str):
        md = list(self.meta)
        if service in self.function_ids:
            md.append(("function-id", self.function_ids[service]))
        return md or None

    def transcribe(self, pcm_chunks, language="en-US", rate=16000):
        cfg = MSG["StreamingRecognitionConfig"](
            config=MSG["RecognitionConfig"](encoding=LINEAR_PCM, sample_rate_hertz=rate, language_code=language,
                                            max_alternatives=1, audio_channel_count=1,
                                            enable_automatic_punctuation=True),
            interim_results=True)

        def reqs():
            yield MSG["StreamingRecognizeRequest"](streaming_config=cfg)
            for c in pcm_chunks:
                if c:
                    yield MSG["StreamingRecognizeRequest"](audio_content=c)

        final = ""
        for resp in self._asr(reqs(), metadata=self._md("asr")):
            partial = ""
            for r in resp.results:
                if not r.alternatives:
                    continue
                if r.is_final:
                    final += r.alternatives[0].transcript
                else:
                    partial += r.alternatives[0].transcript
            yield final + partial

    def synthesize(self, text, language="en-US", voice=""):
        for piece in split_for_tts(text):
            req = MSG["SynthesizeSpeechRequest"](text=piece, language_code=language, encoding=LINEAR_PCM,
                                                 sample_rate_hz=self.sample_rate_tts, voice_name=voice)
            for resp in self._tts(req, metadata=self._md("tts")):
                if resp.audio:
                    yield resp.audio


def backend_from_env() -> SpeechBackend:
    uri = os.environ.get("RIVA_API_URI")
    if not uri:
        return SpeechBackend()
    fids = {k: v for k, v in (("asr", os.environ.get("RIVA_ASR_FUNCTION_ID")),
                              ("tts", os.environ.get("RIVA_TTS_FUNCTION_ID"))) if v}
    return RivaBackend(uri, os.environ.get("RIVA_USE_SSL", "0") == "1", os.environ.get("RIVA_API_KEY"), fids)


def pcm_chunks(pcm: bytes, rate: int = 16000, ms: int = 100) -> Iterator[bytes]:
    step = rate * 2 * ms // 1000
    for i in range(0, len(pcm), step):
        yield pcm[i:i + step]


def tone(freq: float, seconds: float, rate: int) -> bytes:
    """A sine tone as int16 PCM (test fixtures)."""
    import math

    n = int(seconds * rate)
    return b"".join(struct.pack("<h", int(8000 * math.sin(2 * math.pi * freq * i / rate))) for i in range(n))
