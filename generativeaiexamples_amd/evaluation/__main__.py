"""CLI with the reference's flags (rag_evaluator/main.py:27-81, synthetic_data_generator/main.py):

  python -m generativeaiexamples_amd.evaluation --base_url localhost:8081 --generate_answer True \\
      --docs dataset/ --ga_input qa.json --ga_output eval.json
  python -m generativeaiexamples_amd.evaluation --ev_input eval.json --ev_result results/ragas --metrics ragas
  python -m generativeaiexamples_amd.evaluation --ev_input eval.json --ev_result results/judge --metrics judge_llm \\
      --judge_base_url localhost:8000 --judge_llm_model mistralai/mixtral-8x7b-instruct-v0.1
  python -m generativeaiexamples_amd.evaluation --generate_synthetic True --docs dataset/ --sd_output qa.json \\
      --judge_base_url localhost:8000
"""
from __future__ import annotations

import argparse
import json
import logging


def _bool(v):
    return str(v).lower() in ("1", "true", "yes", "y", "")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--base_url", type=str, default="localhost:8081", help="chain server host:port")
    ap.add_argument("--generate_answer", type=_bool, nargs="?", const=True, default=False)
    ap.add_argument("--evaluate", type=_bool, nargs="?", const=True, default=True)
    ap.add_argument("--generate_synthetic", type=_bool, nargs="?", const=True, default=False)
    ap.add_argument("--docs", type=str, default="")
    ap.add_argument("--ga_input", type=str, default="", help="QA JSON, or a ground-truth .txt in the medical-device "
                    "example's 'Example n: / Question: / Answer:' format")
    ap.add_argument("--ga_output", type=str, default="")
    ap.add_argument("--sd_output", type=str, default="qa_generation.json")
    ap.add_argument("--ev_input", type=str, default="")
    ap.add_argument("--ev_result", type=str, default="results/eval")
    ap.add_argument("--metrics", choices=["ragas", "judge_llm"], default="judge_llm")
    ap.add_argument("--judge_llm_model", type=str, default="mistralai/mixtral-8x7b-instruct-v0.1")
    ap.add_argument("--judge_base_url", type=str, default="localhost:8000", help="/v1 server for the judge / generator")
    ap.add_argument("--embedding_model", type=str, default="nvidia/nv-embedqa-e5-v5")
    ap.add_argument("--no_embeddings", action="store_true", help="lexical answer similarity/relevancy only")
    ap.add_argument("--lexical_ragas", action="store_true",
                    help="ragas metrics from word overlap instead of the judge LLM (no model server needed)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from .llm import ChatFn

    if a.generate_synthetic:
        from .synthetic_qa import generate_synthetic_data
        generate_synthetic_data(a.docs, a.sd_output, ChatFn(a.judge_base_url, a.judge_llm_model, temperature=0.2))
    if a.generate_answer:
        from .answer_generator import generate_answers
        qa_file = a.ga_input
        if qa_file.endswith(".txt"):
            from ..examples.medical_device import parse_gt_qa_txt
            qa_file = a.ga_input[:-4] + ".json"
            with open(a.ga_input, encoding="utf-8") as f, open(qa_file, "w", encoding="utf-8") as g:
                json.dump(parse_gt_qa_txt(f.read()), g, indent=2)
        generate_answers(a.base_url, a.docs or None, qa_file, a.ga_output)
    if a.evaluate and a.ev_input:
        import os
        os.makedirs(os.path.dirname(a.ev_result) or ".", exist_ok=True)
        if a.metrics == "ragas":
            from .metrics import eval_ragas
            embed = None
            if not a.no_embeddings:
                from ..chain_server.connectors import RemoteEmbeddings
                re_ = RemoteEmbeddings(a.judge_base_url if a.judge_base_url.startswith("http") else
                                       "http://" + a.judge_base_url, a.embedding_model)
                embed = re_.embed_documents
            judge = None if a.lexical_ragas else ChatFn(a.judge_base_url, a.judge_llm_model, temperature=0.0,
                                                         max_tokens=512)
            print(json.dumps(eval_ragas(a.ev_input, a.ev_result, embed=embed, llm=judge)))
        else:
            from .judge import eval_llm_judge
            res = eval_llm_judge(a.ev_input, a.ev_result, ChatFn(a.judge_base_url, a.judge_llm_model, max_tokens=200))
            print(json.dumps({k: v for k, v in res.items() if k != "rows"}))


if __name__ == "__main__":
    main()
