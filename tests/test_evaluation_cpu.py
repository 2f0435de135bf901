"""Evaluation tool (T1-T3 + load generator) on the CPU plumbing configuration."""
import json
import os

import pytest

from generativeaiexamples_amd.evaluation import judge, metrics, synthetic_qa

REF_QNA = "/root/reference/RAG/tools/evaluation/results/qna.json"


def test_parse_pairs_json_and_regex():
    js = '[{"question": "Who?", "answer": "Ada."}, {"question": "When?", "answer": "1843."}]'
    assert [p["answer"] for p in synthetic_qa.parse_pairs(js)] == ["Ada.", "1843."]
    loose = 'Sure! {"question": "What is HBM?", "answer": "High \\"bandwidth\\" memory"} and more'
    assert synthetic_qa.parse_pairs(loose) == [{"question": "What is HBM?", "answer": 'High "bandwidth" memory'}]


def test_metrics_separate_good_and_bad_answers():
    ctx = "The MI355X accelerator has 288 GB of HBM3E memory. Its wavefronts are 64 lanes wide."
    good = {"question": "How much HBM3E memory does the MI355X have?", "answer": "The MI355X has 288 GB of HBM3E memory.",
            "contexts": [ctx], "gt_answer": "It has 288 GB of HBM3E memory.", "gt_context": ctx}
    bad = dict(good, answer="Bananas grow in tropical climates near rivers.", contexts=["Unrelated text about cooking pasta."])
    g, b = metrics.score_row(good), metrics.score_row(bad)
    assert g["faithfulness"] == 1.0 and g["context_recall"] == 1.0 and g["context_precision"] == 1.0
    assert b["faithfulness"] == 0.0 and b["context_recall"] == 0.0 and b["ragas_score"] == 0.0
    assert g["ragas_score"] > 0.5 and g["answer_similarity"] > b["answer_similarity"]
    emb = lambda texts: [[1.0, 0.0] if "288" in t else [0.0, 1.0] for t in texts]  # noqa: E731
    assert metrics.score_row(good, embed=emb)["answer_similarity"] == 1.0


@pytest.mark.skipif(not os.path.exists(REF_QNA), reason="reference fixture not present")
def test_eval_ragas_on_reference_fixture(tmp_path):
    """The reference's own QnA fixture, answered with its ground truth and retrieving its ground-truth
    context: a perfect pipeline must score recall/faithfulness ~1 (parity with ragas unpinned)."""
    with open(REF_QNA) as f:
        data = json.load(f)[:20]
    rows = [{"question": d["question"], "answer": d["ground_truth_answer"], "contexts": [d["ground_truth_context"]],
             "gt_answer": d["ground_truth_answer"], "gt_context": d["ground_truth_context"]} for d in data]
    p = tmp_path / "ev.json"
    p.write_text(json.dumps(rows))
    agg = metrics.eval_ragas(str(p), str(tmp_path / "res"))
    assert agg["context_precision"] > 0.95 and agg["context_recall"] > 0.7 and agg["faithfulness"] > 0.7
    assert set(metrics.METRIC_NAMES) <= set(agg) and (tmp_path / "res.rows.json").exists()


def test_llm_judge_parsing_and_mean(tmp_path):
    replies = iter(['{"Rating": 5, "Explanation": "correct"}', 'Rating: 0 - wrong', "no idea"])
    rows = [{"question": f"q{i}", "answer": "a", "gt_answer": "a", "gt_context": "c"} for i in range(3)]
    p = tmp_path / "ev.json"
    p.write_text(json.dumps(rows))
    out = judge.eval_llm_judge(str(p), str(tmp_path / "judge"), lambda msgs: next(replies))
    assert [r["rating"] for r in out["rows"]] == [5, 1, None]
    assert out["num_ratings"] == 2 and out["mean_rating"] == 3.0


def test_synthetic_answers_and_load_generator(tmp_path):
    """T1 -> T2 -> T3 + load generator against the real chain-server app (tiny CPU models)."""
    env = {"APP_ENGINE_LLM": "tiny-llama", "APP_ENGINE_EMBEDDER": "tiny-e5", "APP_ENGINE_DEVICE": "cpu",
           "APP_ENGINE_RERANKER": "tiny-reranker", "APP_RETRIEVER_SCORETHRESHOLD": "-1",
           "EXAMPLE_PATH": "basic_rag/langchain", "UPLOAD_DIR": str(tmp_path / "up"), "GAI_LAZY_EXAMPLE": "1",
           "PROMPT_CONFIG_FILE": str(tmp_path / "none.yaml"), "APP_CONFIG_FILE": str(tmp_path / "none.json")}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        from fastapi.testclient import TestClient

        from generativeaiexamples_amd.chain_server import server, utils, vectorstore
        from generativeaiexamples_amd.evaluation.answer_generator import generate_answers
        from generativeaiexamples_amd.evaluation.load_generator import run_load
        from generativeaiexamples_amd.playground import ChatClient

        utils.get_config.cache_clear()
        utils.get_prompts.cache_clear()
        utils.set_hub(None)
        vectorstore.reset_stores()
        server.app.state.example = None
        docs = tmp_path / "docs"
        docs.mkdir()
        (docs / "a.txt").write_text("The MI355X has 288 GB of HBM3E memory per GPU. " * 40)
        fake = lambda msgs: '[{"question": "How much memory?", "answer": "288 GB."}]'  # noqa: E731
        qa = synthetic_qa.generate_synthetic_data(str(docs), str(tmp_path / "qa.json"), fake)
        assert qa and qa[0]["gt_answer"] == "288 GB." and qa[0]["document"] == "a.txt"
        with TestClient(server.app) as chain:
            cc = ChatClient("http://testserver", http=chain)
            ev = generate_answers("", str(docs), str(tmp_path / "qa.json"), str(tmp_path / "ev.json"), client=cc,
                                  max_tokens=4)
            assert ev[0]["contexts"] and "288" in ev[0]["contexts"][0]
            agg = metrics.eval_ragas(str(tmp_path / "ev.json"), str(tmp_path / "res"))
            assert 0 <= agg["ragas_score"] <= 1
            load = run_load("http://testserver", "chain", concurrency=2, requests=4, max_tokens=4, http=chain)
            assert load["requests"] == 4 and load["errors"] == 0 and load["qps"] > 0
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        from generativeaiexamples_amd.chain_server import utils
        utils.get_config.cache_clear()
        utils.set_hub(None)


def _scripted_judge():
    """A deterministic judge implementing each ragas prompt by word overlap (stands in for the LLM)."""
    import re as _re

    from generativeaiexamples_amd.evaluation import ragas_llm as R

    def words(t):
        return set(_re.findall(r"[a-z0-9]+", t.lower())) - {"the", "a", "of", "is", "it", "has"}

    def field(user, name):
        m = _re.search(rf"{name}:\s*(.*?)(?:\n+(?:Question|Answer|Context|Statements|Return)\b|\Z)", user, _re.S)
        return m.group(1).strip() if m else ""

    def fn(messages, schema=None):
        user = messages[-1]["content"]
        items = [ln[2:] for ln in user.split("\n") if ln.startswith("- ")]
        ctx = field(user, "Context")
        if schema is R.S_STATEMENTS:
            return json.dumps({"statements": R.sentences(field(user, "Answer"))})
        if schema is R.S_VERDICTS:
            return json.dumps({"verdicts": [{"statement": s, "verdict": int(words(s) <= words(ctx))} for s in items]})
        if schema is R.S_QUESTION:
            a = field(user, "Answer")
            return json.dumps({"question": a.split("(variant")[0], "noncommittal": int("don't know" in a)})
        if schema is R.S_VERDICT:
            c, a = words(field(user, "Context")), words(field(user, "Answer"))
            return json.dumps({"reason": "", "verdict": int(len(c & a) >= 0.5 * len(a))})
        if schema is R.S_ATTRIB:
            return json.dumps({"classifications": [{"statement": s, "attributed": int(words(s) <= words(ctx))}
                                                   for s in items]})
        if schema is R.S_SENTENCES:
            q = words(field(user, "Question"))
            return json.dumps({"sentences": [s for s in R.sentences(ctx) if len(words(s) & q) >= 2]})
        raise AssertionError(schema)

    return fn


def test_ragas_llm_algorithms_with_scripted_judge(tmp_path):
    from generativeaiexamples_amd.evaluation.ragas_llm import RagasJudge

    ctx1 = "The MI355X has 288 GB of HBM3E memory. Wavefronts are 64 lanes wide."
    ctx2 = "Pasta cooks in salted boiling water."
    emb = lambda texts: [[1.0, 0.2] if "MI355X" in t else [0.1, 1.0] for t in texts]  # noqa: E731
    j = RagasJudge(_scripted_judge(), emb, n_questions=2)
    row = {"question": "How much HBM3E memory does the MI355X have?",
           "answer": "The MI355X has 288 GB of HBM3E memory. It was made of cheese.",
           "contexts": [ctx2, ctx1], "gt_answer": "The MI355X has 288 GB of HBM3E memory."}
    s = j.score_row(row)
    assert s["faithfulness"] == 0.5                 # one of two statements supported
    assert s["context_precision"] == 0.5            # useful context at rank 2 only: P@2 = 1/2
    assert s["context_recall"] == 1.0
    assert abs(s["context_relevancy"] - 1 / 3) < 1e-9  # 1 of 3 context sentences extracted
    assert s["answer_similarity"] > 0.99 and s["answer_relevancy"] > 0.99 and 0 < s["ragas_score"] < 1
    vague = j.score_row(dict(row, answer="I don't know."))
    assert vague["answer_relevancy"] == 0.0 and vague["ragas_score"] == 0.0
    p = tmp_path / "ev.json"
    p.write_text(json.dumps([row]))
    agg = metrics.eval_ragas(str(p), str(tmp_path / "res"), embed=emb, llm=_scripted_judge())
    assert agg["faithfulness"] == 0.5 and agg["context_precision"] == 0.5


def test_ragas_llm_judge_on_served_model_always_parses():
    """The judge runs on our model server with response_format json_schema: constrained decoding makes every
    reply valid JSON of the requested shape even from a random-weight model."""
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.evaluation import ragas_llm as R
    from generativeaiexamples_amd.evaluation.llm import ChatFn
    from generativeaiexamples_amd.serving.hub import HubSpec, ServiceHub
    from generativeaiexamples_amd.serving.openai_api import create_openai_app

    hub = ServiceHub.build(HubSpec(llm="tiny-llama", embedder=None, device="cpu", max_num_seqs=8, max_model_len=1024,
                                   use_graphs=False))
    try:
        with TestClient(create_openai_app(hub)) as c:
            judge = ChatFn("http://testserver", "tiny", temperature=0.7, max_tokens=64, http=c)
            replies = []

            def logged(messages, schema=None):
                r = judge(messages, schema=schema)
                replies.append((schema, r))
                return r

            s = R.RagasJudge(logged, None).score_row(
                {"question": "What is HBM?", "answer": "High bandwidth memory. It is fast.",
                 "contexts": ["HBM is high bandwidth memory."], "gt_answer": "High bandwidth memory."})
            assert all(0.0 <= v <= 1.0 for v in s.values())
            assert len(replies) >= 4
            for schema, r in replies:
                obj = json.loads(r)
                assert set(schema["required"]) <= set(obj)
    finally:
        hub.shutdown()
