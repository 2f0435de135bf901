"""Host timeline of the engine's pipelined multi-step decode (the bench's decode phase): per 8-step run, how long
the chained launch (_chain -> _exec_multi, incl. the graph replay call) and the completion (_complete: token wait +
processing) take on the host, against the GPU time of a run. Llama-3-8B, B sequences of P prompt tokens.

python tools/microbench/decode_host_timeline.py [--batch 64 --prompt 2400 --tokens 96]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams  # noqa: E402
from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer  # noqa: E402
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=2400)
    ap.add_argument("--tokens", type=int, default=96)
    ap.add_argument("--decode-steps", type=int, default=8)
    a = ap.parse_args()
    cfg = LlamaConfig.llama3_8b()
    m = LlamaModel(cfg, device="cuda").random_init(1)
    tok = llama3_byte_tokenizer(cfg.vocab_size)
    eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=a.batch, max_batched_tokens=16384, prefill_chunk=16384,
                                         max_model_len=a.prompt + a.tokens + 64, decode_steps=a.decode_steps,
                                         kv_memory_fraction=0.5))
    eng.capture_graphs(max_bs=a.batch)
    ev = []

    def wrap(name, fn):
        def w(*x, **k):
            t0 = time.perf_counter()
            r = fn(*x, **k)
            ev.append((name, t0, time.perf_counter()))
            return r
        return w

    eng._chain = wrap("chain", eng._chain)
    eng._complete = wrap("complete", eng._complete)
    eng._launch_multi = wrap("launch_multi", eng._launch_multi)
    for rep in range(2):
        ev.clear()
        g = torch.Generator().manual_seed(rep)
        for i in range(a.batch):
            eng.add_request(torch.randint(10, 5000, (a.prompt,), generator=g).tolist(),
                            SamplingParams(temperature=0.2, top_p=0.7, max_tokens=a.tokens, ignore_eos=True))
        t0 = time.perf_counter()
        steps = []
        while eng.has_work():
            ts = time.perf_counter()
            eng.step()
            steps.append((ts, time.perf_counter()))
        torch.cuda.synchronize()
        total = time.perf_counter() - t0
    base = ev[0][1]
    print(f"total {1e3 * total:.1f} ms, {len(steps)} engine steps", flush=True)
    for name, s, e in ev[-16:]:
        print(f"{name:13s} start {1e3 * (s - base):9.2f} ms  dur {1e3 * (e - s):7.2f} ms", flush=True)
    ch = [e - s for n, s, e in ev if n == "chain"]
    co = [e - s for n, s, e in ev if n == "complete"]
    if ch:
        ch.sort()
        co.sort()
        print(f"chain calls {len(ch)} median {1e3 * ch[len(ch) // 2]:.2f} ms max {1e3 * ch[-1]:.2f}; complete median "
              f"{1e3 * co[len(co) // 2]:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
