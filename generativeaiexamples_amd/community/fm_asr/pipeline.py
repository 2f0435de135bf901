"""SDR -> speech -> text streaming pipeline (the reference's Holoscan application, /root/reference/community/
fm-asr-streaming-rag/sdr-holoscan/app.py and operators.py:76-357): a UDP / TCP receiver accumulates packet payloads
into bursts (header bytes stripped), each burst of complex64 baseband samples runs the GPU signal chain of
``dsp.py`` (low-pass -> FM demodulation -> resampling to 16 kHz with gain), the audio is converted to 16-bit PCM and
buffered in one-second pieces for a speech recogniser, whose transcripts are posted to the chain server's
``/storeStreamingText``.

The recogniser is pluggable (``AsrClient``): the reference streams to a remote Riva service (out of scope
here); ``CallableAsr`` wraps any ``pcm_bytes -> text`` function and ``TranscriptPoster`` forwards the text.
"""
from __future__ import annotations

import json
import logging
import queue
import socket
import threading
import time
import urllib.request
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import torch

from . import dsp

log = logging.getLogger(__name__)


@dataclass
class SdrParams:
    """params.yml of the reference (sensor, network_rx, lowpassfilt, resample sections)."""
    sample_rate: float = 1_000_000.0
    ip_addr: str = "0.0.0.0"
    dst_port: int = 5005
    l4_proto: str = "udp"
    batch_size: int = 500_000  # payload bytes per burst
    header_bytes: int = 8
    max_payload_size: int = 1472
    cutoff: float = 100_000.0
    numtaps: int = 101
    sample_rate_out: float = 16_000.0
    gain: float = 10.0
    pcm_chunk_bytes: int = 2 * 16_000  # one second of 16-bit PCM at 16 kHz

    @classmethod
    def from_yaml(cls, path: str) -> "SdrParams":
        import yaml

        with open(path) as f:
            d = yaml.safe_load(f) or {}
        flat = {}
        for sec, key_map in (("sensor", {"sample_rate": "sample_rate"}),
                             ("network_rx", {k: k for k in ("ip_addr", "dst_port", "l4_proto", "batch_size",
                                                            "header_bytes", "max_payload_size")}),
                             ("lowpassfilt", {"cutoff": "cutoff", "numtaps": "numtaps"}),
                             ("resample", {"sample_rate_out": "sample_rate_out", "gain": "gain"})):
            for k, v in (d.get(sec) or {}).items():
                if k in key_map:
                    flat[key_map[k]] = v
        return cls(**flat)


class SignalChain:
    """The per-burst GPU processing: complex64 samples -> float audio at ``sample_rate_out``."""

    def __init__(self, p: SdrParams, device=None):
        self.p = p
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.taps = dsp.firwin(p.numtaps, p.cutoff, fs=p.sample_rate, window="hamming")
        self.taps_dev = torch.as_tensor(self.taps.astype("float32"), device=self.device)  # uploaded once
        self.up, self.down = dsp.rational_factors(p.sample_rate, p.sample_rate_out)

    def __call__(self, samples: torch.Tensor) -> torch.Tensor:
        x = samples.to(self.device, torch.complex64)
        y = dsp.lowpass(self.taps_dev, x)
        d = dsp.fm_demod(y)
        return dsp.resample_poly(d, self.up, self.down, window="hamming", gain=self.p.gain)

    def pcm(self, samples: torch.Tensor) -> bytes:
        return dsp.float_to_pcm16(self(samples)).cpu().numpy().tobytes()


class AsrClient:
    """Speech recogniser interface: 16-bit mono PCM at 16 kHz in, transcript text (possibly empty) out."""

    def transcribe(self, pcm: bytes) -> str:
        raise NotImplementedError


class CallableAsr(AsrClient):
    def __init__(self, fn: Callable[[bytes], str]):
        self.fn = fn

    def transcribe(self, pcm: bytes) -> str:
        return self.fn(pcm)


class TranscriptPoster:
    """Posts transcripts to a chain server's /storeStreamingText (or hands them to a local callable)."""

    def __init__(self, url: Optional[str] = None, source_id: str = "fm-radio",
                 local: Optional[Callable[[str, str], object]] = None):
        self.url, self.source_id, self.local = url, source_id, local

    def __call__(self, text: str) -> None:
        if not text.strip():
            return
        if self.local is not None:
            self.local(self.source_id, text)
            return
        body = json.dumps({"transcript": text, "source_id": self.source_id}).encode()
        req = urllib.request.Request(self.url, data=body, headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=10):
            pass


@dataclass
class _Burst:
    header: bytearray = field(default_factory=bytearray)
    data: bytearray = field(default_factory=bytearray)


class PacketReceiver:
    """UDP / TCP payload accumulator (BasicNetworkRxOp): strips ``header_bytes`` from each packet and emits a burst
    once ``batch_size`` payload bytes have arrived (whole complex64 samples)."""

    def __init__(self, p: SdrParams):
        self.p = p
        self.burst = _Burst()
        self.sock: Optional[socket.socket] = None
        self.conn: Optional[socket.socket] = None

    def open(self) -> int:
        if self.p.l4_proto == "udp":
            self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM, socket.IPPROTO_UDP)
            self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 49_000_000)
        else:
            self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM, socket.IPPROTO_TCP)
        self.sock.bind((self.p.ip_addr, self.p.dst_port))
        if self.p.l4_proto != "udp":
            self.sock.listen(1)
        return self.sock.getsockname()[1]

    def feed(self, packet: bytes) -> Optional[np.ndarray]:
        """Add one packet; returns a complete burst (complex64 samples) when one is ready."""
        self.burst.header.extend(packet[: self.p.header_bytes])
        self.burst.data.extend(packet[self.p.header_bytes:])
        if len(self.burst.data) < self.p.batch_size:
            return None
        n = len(self.burst.data) // 8 * 8
        out = np.frombuffer(bytes(self.burst.data[:n]), dtype=np.complex64).copy()
        rest = self.burst.data[n:]
        self.burst = _Burst(data=bytearray(rest))
        return out

    def receive(self, timeout: float = 1.0) -> Optional[np.ndarray]:
        """Block for packets until a burst is complete (None on timeout)."""
        deadline = time.time() + timeout
        if self.p.l4_proto != "udp" and self.conn is None:
            self.sock.settimeout(timeout)
            try:
                self.conn, _ = self.sock.accept()
            except socket.timeout:
                return None
        src = self.sock if self.p.l4_proto == "udp" else self.conn
        while time.time() < deadline:
            src.settimeout(max(1e-3, deadline - time.time()))
            try:
                pkt = src.recv(self.p.max_payload_size + self.p.header_bytes)
            except socket.timeout:
                return None
            if not pkt:
                return None
            burst = self.feed(pkt)
            if burst is not None:
                return burst
        return None

    def close(self):
        for s in (self.conn, self.sock):
            if s is not None:
                s.close()


class SdrPipeline:
    """Bursts -> signal chain -> one-second PCM pieces -> recogniser (on its own thread) -> transcript sink."""

    def __init__(self, p: SdrParams, asr: AsrClient, sink: Callable[[str], None], device=None):
        self.p, self.asr, self.sink = p, asr, sink
        self.chain = SignalChain(p, device)
        self.pcm = bytearray()
        self.q: "queue.Queue[Optional[bytes]]" = queue.Queue(maxsize=64)
        self.worker = threading.Thread(target=self._asr_loop, daemon=True)
        self.worker.start()
        self.errors = 0

    def process_burst(self, samples) -> int:
        """Run one burst through the signal chain; returns the PCM bytes produced."""
        t = torch.from_numpy(np.asarray(samples, dtype=np.complex64)) if not torch.is_tensor(samples) else samples
        pcm = self.chain.pcm(t)
        self.pcm.extend(pcm)
        while len(self.pcm) >= self.p.pcm_chunk_bytes:
            self.q.put(bytes(self.pcm[: self.p.pcm_chunk_bytes]))
            del self.pcm[: self.p.pcm_chunk_bytes]
        return len(pcm)

    def _asr_loop(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            try:
                self.sink(self.asr.transcribe(item))
            except Exception as e:  # a failed piece is logged and dropped; the stream goes on
                self.errors += 1
                log.warning("asr / sink failed: %s", e)

    def close(self, flush: bool = True):
        if flush and self.pcm:
            self.q.put(bytes(self.pcm))
            self.pcm = bytearray()
        self.q.put(None)
        self.worker.join(timeout=30)

    def run(self, receiver: PacketReceiver, stop: threading.Event):
        while not stop.is_set():
            burst = receiver.receive(timeout=0.5)
            if burst is not None:
                self.process_burst(burst)
