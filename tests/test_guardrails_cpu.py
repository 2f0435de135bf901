"""Parallel guardrails (W10): input rails run concurrently and block, output rails stop the stream."""
import threading
import time

from generativeaiexamples_amd.rag.guardrails import Guardrails, llm_rail


def test_input_rails_parallel_and_blocking():
    active, peak = [0], [0]
    lock = threading.Lock()

    def slow_rail(ok):
        def r(text):
            with lock:
                active[0] += 1
                peak[0] = max(peak[0], active[0])
            time.sleep(0.2)
            with lock:
                active[0] -= 1
            return ok
        return r

    g = Guardrails(input_rails={"safety": slow_rail(True), "topic": slow_rail(False)})
    t0 = time.perf_counter()
    assert g.check_input("how do I bake bread?") == "topic"
    assert time.perf_counter() - t0 < 0.35 and peak[0] == 2  # both rails ran at the same time
    assert list(g.generate("q", lambda: iter(["never"]))) == [g.refusal]


def test_output_rails_windowed_stream():
    g = Guardrails(output_rails={"safety": lambda w: "BAD" not in w}, chunk=10, context=3)
    good = "".join(g.guard_stream(iter(["hello ", "world, this ", "is fine"])))
    assert good == "hello world, this is fine"
    out = list(g.guard_stream(iter(["0123456789", "abcdefBAD", "more text"])))
    assert out[0] == "0123456789" and out[-1].endswith(g.refusal) and "BAD" not in "".join(out)


def test_llm_rail_parses_one_word_answers():
    class L:
        def __init__(self, a):
            self.a = a

        def invoke(self, msgs):
            return self.a
    assert llm_rail(L("Safe."), "p")("x") and not llm_rail(L("unsafe"), "p")("x")
    assert llm_rail(L("on-topic"), "p")("x") and not llm_rail(L(""), "p")("x")
