"""Retriever SDG pipeline: QA parsing, easiness / answerability filters, BEIR export and the IR
metrics, end to end on CPU with a tiny in-process embedder and a scripted LLM."""
import json
import math
import os
import zlib

import numpy as np
import pytest

from generativeaiexamples_amd.evaluation import retriever_sdg as sdg

REF_DATA = "/root/reference/nemo/retriever-synthetic-data-generation/data"


def test_ir_metrics_hand_computed():
    qrels = {"q1": {"d1": 1, "d4": 1}, "q2": {"d9": 1}}
    results = {"q1": {"d1": 0.9, "d2": 0.8, "d4": 0.7, "d5": 0.1}, "q2": {"d3": 0.5, "d2": 0.4}}
    m = sdg.ir_metrics(results, qrels, k_values=(1, 3))
    # q1: hits at ranks 1 and 3; q2: none
    ndcg3_q1 = (1 + 1 / math.log2(4)) / (1 + 1 / math.log2(3))
    assert m["NDCG"]["NDCG@3"] == pytest.approx(ndcg3_q1 / 2, abs=1e-5)
    assert m["Recall"]["Recall@1"] == pytest.approx(0.25)
    assert m["Recall"]["Recall@3"] == pytest.approx(0.5)
    assert m["P"]["P@3"] == pytest.approx((2 / 3) / 2, abs=1e-5)
    assert m["MAP"]["MAP@3"] == pytest.approx(((1 + 2 / 3) / 2) / 2, abs=1e-5)


def test_parse_qa_blocks_reference_style():
    reply = ("Question: When was season four ordered?\nAnswer: On February 5, 2015.\nExplanation: specific.\n\n"
             "Question 2: How many episodes?\nAnswer 2: 23 episodes.\n")
    qas = sdg.parse_qa_blocks(reply)
    assert [q["question"] for q in qas] == ["When was season four ordered?", "How many episodes?"]
    assert qas[0]["answers"][0]["text"] == "On February 5, 2015." and qas[0]["synthetic"]


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference sample data not mounted")
def test_loads_reference_sample_formats():
    c = sdg.Corpus.load(os.path.join(REF_DATA, "sample_data_squad.json"), "squad")
    assert sum(1 for _ in c.paragraphs()) >= 1
    r = sdg.Corpus.load(os.path.join(REF_DATA, "sample_data_rawdoc.jsonl"), "rawdoc")
    assert all(p["context"] and p["document_id"] for p in r.paragraphs())


def _hash_embed(dim=64):
    """Bag-of-words hashing embedder: deterministic, so lexical overlap -> cosine."""
    def fn(texts, input_type):
        out = np.zeros((len(texts), dim), np.float32)
        for i, t in enumerate(texts):
            for w in t.lower().split():
                out[i, zlib.crc32(w.strip(".,?").encode()) % dim] += 1.0
        return out / np.maximum(np.linalg.norm(out, axis=1, keepdims=True), 1e-12)
    return fn


def test_pipeline_end_to_end(tmp_path):
    docs = [{"_id": f"doc{i}", "title": f"T{i}", "text": f"Topic{i} alpha{i} beta{i} was founded in {1900 + i} "
                                                          f"by person{i} in city{i}."} for i in range(12)]
    src = tmp_path / "raw.jsonl"
    src.write_text("\n".join(json.dumps(d) for d in docs))

    def llm(messages):
        text = messages[-1]["content"]
        if "criterion" in messages[0]["content"].lower() or "Criterion" in text:
            bad = "person3" in text  # one question judged unanswerable
            return json.dumps({f"criterion_{i}": ("N" if bad and i == 4 else "Y") for i in range(1, 5)})
        i = int(text.split("Topic")[1].split()[0])
        return (f"Question: Who founded topic{i}?\nAnswer: person{i}\nExplanation: ok\n"
                f"Question: What year was alpha{i} started?\nAnswer: {1900 + i}\n")

    embed = _hash_embed()
    gen = sdg.QAGenerator(llm, num_questions=2, max_examples=10)
    filters = [sdg.EasinessFilter(embed, percentile=70), sdg.AnswerabilityFilter(llm)]
    rep = sdg.run_pipeline(sdg.Corpus.load(str(src), "rawdoc"), str(tmp_path / "out"), gen, filters,
                           {"hash": embed})
    assert rep["all"]["questions"] == 20
    assert 0 < rep["filtered"]["questions"] < rep["all"]["questions"]
    all_c = json.load(open(tmp_path / "out/squad/synthetic_data__all.json"))
    qas = [qa for ex in all_c["data"] for qa in ex["paragraphs"][0]["qas"]]
    assert all("easiness__cossim" in qa and "answerability__keep" in qa for qa in qas)
    sims = [qa["easiness__cossim"] for qa in qas]
    thr = np.percentile(sims, 70)
    assert [qa["easiness__keep"] for qa in qas] == [s <= thr for s in sims]
    assert 12 <= sum(qa["easiness__keep"] for qa in qas) < 20
    for name in ("all", "filtered"):
        d = tmp_path / "out/beir" / name / "synthetic"
        assert (d / "corpus.jsonl").exists() and (d / "qrels/test.tsv").exists()
        ev = json.load(open(tmp_path / "out/eval" / name / "beir_evaluator__type_model_eval_dict.json"))
        r5 = ev["synthetic"]["hash"]["recall"]["Recall@5"]
        assert 0.0 <= r5 <= 1.0
    # the lexical embedder finds the source passage for most questions
    assert rep["all"]["eval"]["hash"]["recall"]["Recall@5"] > 0.5


def test_engine_embedder_adapter():
    import torch

    from generativeaiexamples_amd.engine.embedder import Embedder
    from generativeaiexamples_amd.engine.tokenizer import bert_byte_tokenizer
    from generativeaiexamples_amd.models.bert import BertConfig, BertModel

    enc = BertModel(BertConfig.tiny(), device="cpu").random_init(0)
    fn = sdg.engine_embed_fn(Embedder(enc, bert_byte_tokenizer(2048)))
    corpus = {f"d{i}": {"title": "", "text": f"passage number {i}"} for i in range(5)}
    res = sdg.retrieve(fn, corpus, {"q": "passage number 3"}, top_k=3)
    assert len(res["q"]) == 3 and all(np.isfinite(v) for v in res["q"].values())
    del torch
