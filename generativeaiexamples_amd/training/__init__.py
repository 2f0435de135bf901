"""LoRA supervised fine-tuning (SURVEY P2/P3, W1-W5 side workloads: the reference fine-tunes Gemma /
CodeGemma / StarCoder2 with NeMo LoRA and SFT, TP=4 x DP=2, resume_if_exists, then merges the adapter).

* :mod:`.lora` - adapters (A: [r, in] Kaiming, B: [out, r] zero) on the fused QKV / O / gate-up / down
  projections, merge into the base weights, safetensors save/load.
* :mod:`.tp` - autograd-aware tensor-parallel collectives (column-parallel input: identity forward /
  all-reduce backward; row-parallel output: all-reduce forward / identity backward; vocab gather).
* :mod:`.ddp` - gradient bucketer: per-parameter post-accumulate hooks launch async all-reduces of
  ~25 MB flat buckets over the data-parallel group while the backward pass is still running.
* :mod:`.data` - JSONL instruction data (prompt/response or Dolly instruction/context/response),
  chat-templated, loss masked to the response, packed into fixed-length micro-batches.
* :mod:`.trainer` - AdamW + warmup/cosine, grad accumulation and clipping, checkpoint every N steps
  with resume-if-exists, merge-and-export to a HF safetensors directory.
Training compute uses PyTorch autograd ops (hipBLASLt GEMMs, SDPA) on the frozen bf16 base weights;
the HIP inference kernels have no backward pass.
"""
