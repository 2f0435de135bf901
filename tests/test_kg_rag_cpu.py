"""Knowledge-graph RAG community app (reference community/knowledge_graph_rag): triple parsing, the graph
(k-hop facts, GraphML / CSV interchange), document ingest, text / graph / combined answers and the FastAPI backend,
driven by a scripted LLM and a hashing embedder on the CPU."""
import csv
import json
import os
import zlib

import pandas as pd
import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.community.kg_rag import KGRag, KnowledgeGraph, parse_entities, parse_triples
from generativeaiexamples_amd.community.kg_rag.extract import (RELATIONS, TRIPLE_PROMPT, parse_judgement,
                                                               process_documents)

DOCS = {
    "contoso": "Contoso Labs released the Falcon sensor in Norway. The Falcon sensor reduces grid losses.",
    "fabrikam": "Fabrikam invests in Contoso Labs. Alice Smith is a member of Fabrikam.",
}
TRIPLES = {
    "contoso": "Here you go:\n```python\n[('Contoso Labs', 'ORG', 'Introduce', 'Falcon sensor', 'PRODUCT'),\n"
               " ('Contoso Labs', 'ORG', 'Operate_In', 'Norway', 'GPE'),\n"
               " ('Falcon sensor', 'PRODUCT', 'Positive_Impact_On', 'Grid Losses', 'METRIC')]\n```",
    "fabrikam": '[["Fabrikam", "ORG", "Invests_In", "contoso labs", "ORG"], '
                '["Alice Smith", "PERSON", "is member of", "Fabrikam", "ORG"], ["NaN", "ORG", "Has", "X", "ORG"]]',
}


class _HashEmb(Embeddings):
    dim = 64

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().split():
                out[i, zlib.crc32(w.strip(".,?").encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


class _LLM:
    def __init__(self, entity_reply='{"entities": ["Fabrikam"]}'):
        self.entity_reply, self.calls = entity_reply, []

    def invoke(self, messages, **kw):
        sys_, user = messages[0]["content"], messages[-1]["content"]
        self.calls.append(sys_[:24])
        if sys_ == TRIPLE_PROMPT:
            return next((v for k, v in TRIPLES.items() if user.lower().startswith(k)), "[]")
        if "named entities" in sys_:
            return self.entity_reply
        if "hard question" in sys_:
            return 'Sure: {"question": "Who invests in Contoso Labs?", "answer": "Fabrikam"}'
        if "Rate how well" in sys_:
            return "Evaluation: covers it.\nTotal rating: 3"
        return f"ANSWER<{user}>"


def test_parse_triples_formats():
    rows = parse_triples(TRIPLES["contoso"])
    assert [r["relation"] for r in rows] == ["Introduce", "Operate_In", "Positive_Impact_On"]
    assert rows[0] == {"subject": "Contoso Labs", "subject_type": "ORG", "relation": "Introduce",
                       "object": "Falcon sensor", "object_type": "PRODUCT"}
    rows = parse_triples(TRIPLES["fabrikam"])  # JSON lists, a NaN row, a free-form relation
    assert len(rows) == 2 and rows[1]["relation"] == "Is_Member_Of"
    dicts = json.dumps([{"subject": "A Co", "relation": "has", "object": "B Co"}])
    assert parse_triples(dicts)[0]["relation"] == "Has" and parse_triples(dicts)[0]["object_type"] == "Unknown"
    cut = "[('Acme', 'ORG', 'Produce', 'Widgets', 'PRODUCT'), ('Acme', 'ORG', 'Operate_In', 'Ohi"  # truncated reply
    assert [r["object"] for r in parse_triples(cut)] == ["Widgets"]
    assert parse_triples("[('Acme', 'ORG', 'Likes', 'Widgets', 'PRODUCT')]")[0]["relation"] == "Likes"
    assert parse_triples("[('Acme', 'ORG', 'Likes', 'Widgets', 'PRODUCT')]", strict=True) == []
    for junk in ("no triples here", "", None, "[1, 2, 3]", "[('a', 'b')]"):
        assert parse_triples(junk) == []
    assert all(r in TRIPLE_PROMPT for r in RELATIONS)


def _graph():
    g = KnowledgeGraph()
    g.add_triples([("A", "ORG", "Has", "B", "PRODUCT"), ("B", "PRODUCT", "Impact", "C", "METRIC"),
                   ("C", "METRIC", "Relate_To", "D", "CONCEPT"), ("C", None, "Relate_To", "A", None),
                   ("E", "PERSON", "Is_Member_Of", "A", "ORG")])
    return g


def test_graph_entity_knowledge():
    g = _graph()
    assert len(g) == 5 and g.num_edges == 5
    assert not g.add_triple("a", None, "Has", " b ")  # case / whitespace-insensitive duplicate
    assert g.entity_knowledge("a", depth=1) == ["A Has B"]
    assert g.entity_knowledge("A", depth=2) == ["A Has B", "B Impact C"]
    deep = g.entity_knowledge("A", depth=5)  # the C -> A cycle terminates, each edge once
    assert deep == ["A Has B", "B Impact C", "C Relate_To D", "C Relate_To A"]
    assert "E Is_Member_Of A" in g.entity_knowledge("A", depth=1, both_directions=True)
    assert g.entity_knowledge("nobody") == []
    assert g.find_entities("what does a have to do with E?") == []  # single letters never match
    g.add_triple("Contoso Labs", "ORG", "Has", "Contoso", "ORG")
    assert g.find_entities("Is contoso labs bigger than Contoso? (Contosos)") == ["Contoso Labs", "Contoso"]
    assert g.types["c"] == "METRIC"  # a later untyped mention does not erase the type


def test_find_entities_matches_word_bounded_regex():
    """The first-word index + find() lookup gives exactly the word-bounded regex hits, and sees entities added later."""
    import random
    import re

    g = KnowledgeGraph()
    rnd = random.Random(0)
    words = [f"w{i}" for i in range(50)]
    for i in range(300):
        g.add_triple(" ".join(rnd.sample(words, 2)), "T", "rel", f"ent {i}", "T")
    g.add_triple("C++", "Lang", "used_by", "u.s. navy", "Org")
    g.add_triple("(paren) thing", "X", "near", "_under", "X")
    texts = ["about " + " ".join(rnd.sample(words, 12)) + " and C++ at the u.s. navy, ent 17 and (paren) thing _under",
             "ent 12x c++x w1w2 the_under ent 3."]
    for t in texts:
        low = " " + " ".join(t.split()).lower() + " "
        want = {g.names[k] for k in g.names if len(k) > 1 and re.search(r"(?<![\w])" + re.escape(k) + r"(?![\w])", low)}
        got = g.find_entities(t)
        assert set(got) == want and len(got) == len(want)
        assert [len(x) for x in got] == sorted((len(x) for x in got), reverse=True)
    assert "new thing" not in g.find_entities("a new thing")
    g.add_triple("new thing", "T", "rel", "ent 1", "T")  # the index is rebuilt after a new entity
    assert "new thing" in g.find_entities("a new thing")
    assert g.add_triple("new thing", "T", "rel", "ent 1", "T") is False  # duplicate edge


def test_graphml_and_csv_roundtrip(tmp_path):
    g = _graph()
    p = str(tmp_path / "kg.graphml")
    g.write_graphml(p)
    h = KnowledgeGraph.read_graphml(p)
    assert sorted(h.triples()) == sorted(g.triples()) and h.types == g.types
    # a networkx-style file: node ids are names, the relation is a keyed edge attribute, no node types
    nx_file = tmp_path / "nx.graphml"
    nx_file.write_text(
        '<?xml version="1.0" encoding="utf-8"?>\n<graphml xmlns="http://graphml.graphdrawing.org/xmlns">'
        '<key id="d0" for="edge" attr.name="relation" attr.type="string"/><graph edgedefault="directed">'
        '<node id="Apple Inc."/><node id="iPhone 14"/><edge source="Apple Inc." target="iPhone 14">'
        '<data key="d0">Introduce</data></edge></graph></graphml>')
    n = KnowledgeGraph.read_graphml(str(nx_file))
    assert n.entity_knowledge("apple inc.") == ["Apple Inc. Introduce iPhone 14"]
    g.to_csvs(str(tmp_path / "csv"))
    ents = pd.read_csv(tmp_path / "csv" / "entities.csv")
    rels = pd.read_csv(tmp_path / "csv" / "relations.csv")
    tri = pd.read_csv(tmp_path / "csv" / "triples.csv")
    name = ents.set_index("entity_id")["entity_name"].to_dict()
    rel = rels.set_index("relation_id")["relation_name"].to_dict()
    assert sorted((name[a], rel[r], name[b]) for a, r, b in tri.itertuples(index=False)) == sorted(g.triples())


def test_process_documents_builds_graph():
    seen = []
    chunks, g = process_documents(list(DOCS.values()), _LLM(), chunk_size=500, chunk_overlap=100, max_workers=4,
                                  update_progress=lambda d, t: seen.append((d, t)))
    assert len(chunks) == 2 and seen[-1] == (2, 2)
    assert g.num_edges == 5 and "contoso labs" in g  # "contoso labs" merged with "Contoso Labs"
    assert g.entity_knowledge("Fabrikam", depth=2) == [
        "Fabrikam Invests_In Contoso Labs", "Contoso Labs Introduce Falcon sensor", "Contoso Labs Operate_In Norway"]
    assert all("triples" in c.metadata for c in chunks)


def test_parse_entities():
    assert parse_entities('Sure! {"entities": ["A", "B"]}') == ["A", "B"]
    assert parse_entities("['Apple', 'Google']") == ["Apple", "Google"]
    assert parse_entities("I cannot tell.") is None


def _rag(entity_reply='{"entities": ["Fabrikam"]}'):
    chunks, g = process_documents(list(DOCS.values()), _LLM(), max_workers=2)
    store = VectorStore("kg", _HashEmb(), device="cpu", hybrid=True)
    store.add_documents(chunks)
    return KGRag(_LLM(entity_reply), g, store, k=1)


def test_graph_text_and_combined_answers():
    rag = _rag()
    ans, facts = rag.graph_rag("Who does Fabrikam invest in?")
    assert "Fabrikam Invests_In Contoso Labs" in facts and "Fabrikam Invests_In Contoso Labs" in ans
    ans, ps = rag.text_rag("Who invests in Contoso Labs?")
    assert ps == [DOCS["fabrikam"]] and DOCS["fabrikam"] in ans
    out = rag.chat("Who does Fabrikam invest in?")
    assert out["use_kg"] and "Invests_In" in out["context"] and out["assistant_response"].startswith("ANSWER<")
    assert rag.chat("hi", use_kg=False)["context"] == ""
    # an unparseable entity reply falls back to graph names found in the question
    rag = _rag("I cannot tell.")
    assert "Contoso Labs Operate_In Norway" in rag.graph_facts("Where does contoso labs operate?")
    rag = _rag('{"entities": ["Nobody"]}')
    ans, facts = rag.graph_rag("Tell me about Nobody")
    assert facts == ["no relationship found"] and "not grounded" in ans
    row = _rag().evaluate_question("Who does Fabrikam invest in?", "Contoso Labs")
    assert set(row) >= {"textRAG_answer", "graphRAG_answer", "combined_answer", "combined_RAG_context_response"}


def test_judgement_parse():
    assert parse_judgement("Evaluation: ok\nTotal rating: 4") == {"llm_judge_evaluation": "ok", "llm_judge_score": 4.0}
    assert parse_judgement("rubbish")["llm_judge_score"] == 0.0


def _ndjson(resp):
    return [json.loads(line) for line in resp.text.splitlines() if line.strip()]


def test_server_endpoints(tmp_path):
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.community.kg_rag.server import create_app

    docs_dir = tmp_path / "docs"
    docs_dir.mkdir()
    for k, v in DOCS.items():
        (docs_dir / f"{k}.txt").write_text(v)
    data = tmp_path / "data"
    store = VectorStore("kg", _HashEmb(), device="cpu", hybrid=True)
    app = create_app(lambda model_id: _LLM(), store, str(data), models=lambda: ["local-llm"], max_workers=2)
    c = TestClient(app)
    assert c.get("/get-models/").json() == {"models": ["local-llm"]}
    assert c.get("/check-file-exists/").json() == {"file_exists": False}
    assert c.post("/process-documents/", json={"directory": str(tmp_path / "missing"), "model_id": ""}).status_code \
        == 404
    assert c.post("/process-documents/", json={"directory": str(docs_dir), "model_id": "m"}).status_code == 200
    assert c.get("/progress/").json() == {"progress": "1.0"}
    assert c.get("/check-file-exists/").json() == {"file_exists": True}
    assert len(store) == 2 and {"entities.csv", "relations.csv", "triples.csv", "documents.csv"} <= set(os.listdir(data))
    out = c.post("/chat/", json={"user_input": "Who does Fabrikam invest in?", "use_kg": True, "model_id": "m"}).json()
    assert "Fabrikam Invests_In Contoso Labs" in out["context"]
    qa = _ndjson(c.post("/create-qa-pairs/", json={"num_data": 2, "model_id": "m"}))
    assert len(qa) == 2 and qa[0]["answer"] == "Fabrikam"
    with open(data / "qa_data.csv") as f:
        assert len(list(csv.DictReader(f))) == 2
    ev = _ndjson(c.post("/run-evaluation/", json={"questions_list": ["Who does Fabrikam invest in?"],
                                                  "answers_list": ["Contoso Labs"], "model_id": "m"}))
    assert len(ev) == 1 and "Invests_In" in ev[0]["graphRAG_answer"]
    assert os.path.exists(data / "combined_results.csv")
    sc = _ndjson(c.post("/run-scoring_llm_as_a_judge/", json={"combined_results": ev}))
    assert sc[0]["graphRAG_llm_judge_score"] == 3.0 and sc[0]["gt_llm_judge_score"] == 3.0
    assert c.post("/run-scoring/", json={"combined_results": ev}).status_code == 501
    vis = c.get("/visualization", params={"entity": "Fabrikam", "depth": 1}).json()
    assert {e["target"] for e in vis["edges"]} == {"Contoso Labs", "Fabrikam"}
    # a restarted backend re-reads the GraphML
    app2 = create_app(lambda model_id: _LLM(), store, str(data))
    assert app2.state.kg["graph"].num_edges == 5
    assert app2.state.kg["graph"].types["alice smith"] == "PERSON"  # entity types survive the merge + GraphML


@pytest.mark.parametrize("depth", [0, 1, 3])
def test_entity_knowledge_depth_bounds(depth):
    g = KnowledgeGraph()
    for i in range(5):
        g.add_triple(f"n{i}", None, "Relate_To", f"n{i + 1}")
    assert len(g.entity_knowledge("n0", depth=depth)) == depth
