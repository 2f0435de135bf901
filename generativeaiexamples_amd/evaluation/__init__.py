"""RAG evaluation tool (reference RAG/tools/evaluation):

* :mod:`.synthetic_qa` - synthetic question/answer pairs from a document folder (T1);
* :mod:`.answer_generator` - uploads the documents to a chain server and fills answers + retrieved
  contexts for every question (T2);
* :mod:`.metrics` - RAGAS-style metrics (answer similarity, faithfulness, context precision /
  relevancy / recall, answer relevancy, harmonic-mean ``ragas_score``) computed with this
  framework's own embedder + lexical entailment, and :mod:`.judge` - Likert 1-5 LLM judge (T3);
* :mod:`.load_generator` - concurrent streaming load against /generate or /v1/chat/completions
  (QPS, TTFT and inter-token latency percentiles).

``python -m generativeaiexamples_amd.evaluation --help`` mirrors the reference CLI flags.
"""
