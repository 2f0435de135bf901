"""Tokenizers, chat templates and incremental (streaming) detokenisation.

* :class:`HFTokenizer` wraps a local ``tokenizer.json`` (HF ``tokenizers``, Rust-backed) - used
  whenever a model directory with tokenizer files is available.
* :class:`ByteTokenizer` is the offline fallback (no network, no checkpoints): UTF-8 bytes map to
  ids ``offset..offset+255`` and the model family's special tokens keep their real ids, so prompt
  lengths, chat framing and EOS handling behave like the real tokenizer (1 token per byte).
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Optional, Sequence

import numpy as np


class Tokenizer:
    bos_id: Optional[int] = None
    eos_ids: Sequence[int] = ()
    pad_id: int = 0
    vocab_size: int = 0
    special: Dict[str, int] = {}

    def encode(self, text: str, add_special: bool = False) -> List[int]:
        raise NotImplementedError

    def decode(self, ids: Sequence[int]) -> str:
        raise NotImplementedError

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        return self.decode(ids).encode("utf-8")

    def token_id(self, name: str) -> Optional[int]:
        return self.special.get(name)


class ByteTokenizer(Tokenizer):
    def __init__(self, vocab_size: int, offset: int = 0, special: Optional[Dict[str, int]] = None,
                 bos: Optional[str] = None, eos: Sequence[str] = (), pad: Optional[str] = None):
        assert offset + 256 <= vocab_size or vocab_size == 0
        self.vocab_size = vocab_size
        self.offset = offset
        self.special = dict(special or {})
        self.inv_special = {v: k for k, v in self.special.items()}
        self.bos_id = self.special.get(bos) if bos else None
        self.eos_ids = tuple(self.special[e] for e in eos if e in self.special)
        self.pad_id = self.special.get(pad, 0) if pad else 0

    _SPECIAL_START = re.compile(r"[<\[]")

    def _bytes_ids(self, piece: str) -> List[int]:
        raw = piece.encode("utf-8")
        if self.offset == 0:
            return list(raw)
        return (np.frombuffer(raw, np.uint8).astype(np.int32) + self.offset).tolist()

    def encode(self, text: str, add_special: bool = False) -> List[int]:
        ids: List[int] = []
        i, n = 0, len(text)
        if self.special:
            # split on special-token literals present in the text (runs between candidates in one C-level call)
            names = sorted(self.special, key=len, reverse=True)
            while i < n:
                if text[i] == "<" or text[i] == "[":
                    hit = next((nm for nm in names if text.startswith(nm, i)), None)
                    if hit is not None:
                        ids.append(self.special[hit])
                        i += len(hit)
                        continue
                m = self._SPECIAL_START.search(text, i + 1)
                j = m.start() if m else n
                ids.extend(self._bytes_ids(text[i:j]))
                i = j
        else:
            ids = self._bytes_ids(text)
        if add_special and self.bos_id is not None:
            ids = [self.bos_id] + ids
        return ids

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        out = bytearray()
        for t in ids:
            t = int(t)
            if self.offset <= t < self.offset + 256:
                out.append(t - self.offset)
            elif t in self.inv_special:
                continue  # special tokens are not rendered
            else:
                # ids outside the byte range (random-init models emit any id): render a stable byte
                out.append(32 + (t % 95))
        return bytes(out)

    def decode(self, ids: Sequence[int]) -> str:
        return self.decode_bytes(ids).decode("utf-8", errors="replace")


class HFTokenizer(Tokenizer):
    def __init__(self, path: str):
        from tokenizers import Tokenizer as _T

        f = path if path.endswith(".json") else os.path.join(path, "tokenizer.json")
        self.tk = _T.from_file(f)
        self.vocab_size = self.tk.get_vocab_size()
        vocab = self.tk.get_vocab()
        self.special = {t: i for t, i in vocab.items() if t.startswith("<|") or t in ("<s>", "</s>", "[CLS]", "[SEP]")}
        self.bos_id = self.special.get("<|begin_of_text|>", self.special.get("<s>", self.special.get("[CLS]")))
        eos = [self.special.get(n) for n in ("<|end_of_text|>", "<|eot_id|>", "</s>", "[SEP]")]
        self.eos_ids = tuple(e for e in eos if e is not None)
        self.pad_id = vocab.get("[PAD]", vocab.get("<pad>", 0))

    def encode(self, text: str, add_special: bool = False) -> List[int]:
        ids = self.tk.encode(text, add_special_tokens=False).ids
        if add_special and self.bos_id is not None:
            ids = [self.bos_id] + ids
        return ids

    def decode(self, ids: Sequence[int]) -> str:
        return self.tk.decode(list(map(int, ids)), skip_special_tokens=True)


# ----------------------------------------------------------------------------------- families
LLAMA3_SPECIAL = {
    "<|begin_of_text|>": 128000, "<|end_of_text|>": 128001, "<|start_header_id|>": 128006,
    "<|end_header_id|>": 128007, "<|eot_id|>": 128009, "<|eom_id|>": 128008, "<|python_tag|>": 128010,
}


def llama3_byte_tokenizer(vocab_size: int = 128256) -> ByteTokenizer:
    return ByteTokenizer(vocab_size, 0, LLAMA3_SPECIAL, bos="<|begin_of_text|>", eos=("<|end_of_text|>", "<|eot_id|>"))


def bert_byte_tokenizer(vocab_size: int = 30522) -> ByteTokenizer:
    sp = {"[PAD]": 0, "[UNK]": 100, "[CLS]": 101, "[SEP]": 102, "[MASK]": 103}
    return ByteTokenizer(vocab_size, 1000, sp, bos="[CLS]", eos=("[SEP]",), pad="[PAD]")


def small_byte_tokenizer(vocab_size: int = 512) -> ByteTokenizer:
    sp = {"<s>": 1, "</s>": 2, "<|start_header_id|>": 3, "<|end_header_id|>": 4, "<|eot_id|>": 5}
    return ByteTokenizer(vocab_size, 8, sp, bos="<s>", eos=("</s>", "<|eot_id|>"))


def load_tokenizer(path: Optional[str], family: str = "llama3", vocab_size: Optional[int] = None) -> Tokenizer:
    if path and (os.path.isfile(path) or os.path.isfile(os.path.join(path, "tokenizer.json"))):
        return HFTokenizer(path)
    if family == "bert":
        return bert_byte_tokenizer(vocab_size or 30522)
    if family == "llama3" and (vocab_size is None or vocab_size >= 128256):
        return llama3_byte_tokenizer(vocab_size or 128256)
    return small_byte_tokenizer(vocab_size or 512)


# ----------------------------------------------------------------------------------- chat templates
def image_token_of(model) -> Optional[int]:
    """The image placeholder token id of a multimodal generator (Mllama's <|image|>), None for text models."""
    return getattr(getattr(model, "mcfg", None), "image_token_id", None)


def apply_chat_template(messages: List[dict], tok: Tokenizer, add_generation_prompt: bool = True,
                        image_token_id: Optional[int] = None) -> List[int]:
    """Llama-3 chat format when its header tokens exist, else a plain role-prefixed format. A list content holds
    OpenAI-style parts: text parts are encoded in order; image parts (``image_url`` / ``image``) become
    ``image_token_id`` where they stand (Llama-3.2-Vision's <|image|>) when one is given, else they are dropped."""
    sh, eh, eot = tok.token_id("<|start_header_id|>"), tok.token_id("<|end_header_id|>"), tok.token_id("<|eot_id|>")
    ids: List[int] = []
    if tok.bos_id is not None:
        ids.append(tok.bos_id)

    def body(content) -> List[int]:
        if not isinstance(content, list):
            return tok.encode("\n\n" + (content or "").strip())
        out, first_text = tok.encode("\n\n"), True
        for p in content:
            if not isinstance(p, dict):
                continue
            if p.get("type") in ("image_url", "image"):
                if image_token_id is not None:
                    out.append(image_token_id)
            elif p.get("type") in ("text", None):
                t = p.get("text", "")
                out += tok.encode(t.lstrip() if first_text else t)
                first_text = False
        return out

    if sh is not None and eh is not None and eot is not None:
        for m in messages:
            ids += [sh] + tok.encode(m.get("role", "user")) + [eh] + body(m.get("content")) + [eot]
        if add_generation_prompt:
            ids += [sh] + tok.encode("assistant") + [eh] + tok.encode("\n\n")
        return ids
    if image_token_id is not None and any(isinstance(m.get("content"), list) and any(
            isinstance(p, dict) and p.get("type") in ("image_url", "image") for p in m["content"]) for m in messages):
        ids.append(image_token_id)
    messages = [dict(m, content="".join(p.get("text", "") for p in m["content"] if isinstance(p, dict))
                     if isinstance(m.get("content"), list) else m.get("content")) for m in messages]
    text = "".join(f"{m.get('role', 'user')}: {m.get('content') or ''}\n" for m in messages)
    if add_generation_prompt:
        text += "assistant: "
    return ids + tok.encode(text)


class IncrementalDetokenizer:
    """Streams text deltas for a growing id list; never splits a UTF-8 sequence or a stop string."""

    def __init__(self, tok: Tokenizer, stop: Sequence[str] = ()):
        self.tok = tok
        self.ids: List[int] = []
        self.sent = 0  # chars already emitted
        self.text = ""
        self.stop = [s for s in stop if s]
        self.hold = max((len(s) for s in self.stop), default=1) - 1
        self.stopped = False

    def _decode(self) -> str:
        raw = self.tok.decode_bytes(self.ids) if self.ids else b""
        # only decode complete UTF-8 sequences
        cut = len(raw)
        for back in range(1, min(4, len(raw)) + 1):
            b = raw[-back]
            if b & 0xC0 == 0x80:
                continue
            need = 2 if b & 0xE0 == 0xC0 else 3 if b & 0xF0 == 0xE0 else 4 if b & 0xF8 == 0xF0 else 1
            if need > back:
                cut = len(raw) - back
            break
        return raw[:cut].decode("utf-8", errors="replace")

    def prime(self, ids: Sequence[int], sent_chars: Optional[int] = None) -> None:
        """Continue a completion another replica started (elastic re-queue): ``ids`` were generated there and
        ``sent_chars`` characters of their text already reached the client (default: all complete ones)."""
        for t in ids:
            self.ids.append(int(t))
        self.text = self._decode()
        self.sent = len(self.text) if sent_chars is None else min(int(sent_chars), len(self.text))

    def add(self, token: int) -> str:
        if self.stopped:
            return ""
        self.ids.append(int(token))
        self.text = self._decode()
        for s in self.stop:
            k = self.text.find(s, max(0, self.sent - len(s)))
            if k >= 0:
                self.text = self.text[:k]
                self.stopped = True
                break
        limit = len(self.text) if self.stopped else max(self.sent, len(self.text) - self._partial_stop())
        delta = self.text[self.sent:limit]
        self.sent = limit
        return delta

    def _partial_stop(self) -> int:
        """Characters to hold back: the longest unsent suffix of the text that begins a stop string (a stop
        string may still complete there). Everything before it streams now - a fixed hold of the longest
        stop string's length would delay the first frame by several tokens (behind a whole prefill wave)."""
        t, lo = self.text, self.sent
        for k in range(min(self.hold, len(t) - lo), 0, -1):
            tail = t[len(t) - k:]
            if any(s.startswith(tail) for s in self.stop):
                return k
        return 0

    def flush(self) -> str:
        delta = self.text[self.sent:]
        self.sent = len(self.text)
        return delta
