"""LoRA SFT on the GPU (bf16 base weights, hipBLASLt GEMMs + SDPA under autograd)."""
import pytest
import torch

from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
from generativeaiexamples_amd.parallel.dist import DistContext
from generativeaiexamples_amd.training.lora import LoRAConfig
from generativeaiexamples_amd.training.trainer import LoRATrainer, TrainConfig

pytestmark = pytest.mark.gpu


def test_lora_sft_gpu_loss_falls(cuda):
    ctx = DistContext(device=torch.device("cuda", 0))
    m = LlamaModel(LlamaConfig.tiny(num_layers=2), device="cuda", dist_ctx=ctx).random_init(seed=3)
    tr = LoRATrainer(m, small_byte_tokenizer(m.cfg.vocab_size), LoRAConfig(r=8, alpha=16, targets=("qkv", "o", "gate_up", "down")),
                     TrainConfig(steps=20, global_batch=8, micro_batch=4, seq_len=128, lr=3e-3, warmup=2,
                                 checkpoint_activations=True))
    h = tr.train()
    assert all(x == x for x in h) and h[-1] < 0.5 * h[0]
    assert tr.lora.params["l0.qkv.A"].device.type == "cuda"


def test_embed_finetune_on_gpu(cuda):
    """Contrastive full-weight fine-tuning on the GPU (bf16 autocast), then the tuned weights serve through
    the HIP encoder kernels and agree with the training forward."""
    from generativeaiexamples_amd.engine.embedder import Embedder
    from generativeaiexamples_amd.engine.tokenizer import bert_byte_tokenizer
    from generativeaiexamples_amd.models.bert import BertConfig, BertModel
    from generativeaiexamples_amd.training import embed_ft as E

    torch.manual_seed(0)
    enc = BertModel(BertConfig.tiny(num_layers=2), device=cuda).random_init(3)
    emb = Embedder(enc, bert_byte_tokenizer(2048))
    rows = E.synthetic_pairs(64)
    before = E.recall_at_k(emb, rows[:32])
    ft = E.EmbedFineTuner(emb, E.EmbedFTConfig(global_batch=16, micro_batch=8, lr=3e-4, max_steps=20, tau=0.05), rows)
    hist = ft.fit()
    assert sum(hist[-4:]) < sum(hist[:4])
    assert E.recall_at_k(emb, rows[:32]) >= before
    texts = ["query: w1 w2 w3", "passage: some passage text"]
    with torch.no_grad():
        train_side = ft._encode(texts, "passage").float()
    serve_side = emb.embed(texts, "passage").float()
    torch.testing.assert_close(train_side, serve_side, rtol=0, atol=5e-2)


def test_full_weight_pretrain_gpu(cuda):
    """From-scratch pretraining of a small Llama in bf16 on the GPU (fp32 masters + AdamW): loss falls."""
    import torch

    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.parallel.dist import DistContext
    from generativeaiexamples_amd.rag import synthetic
    from generativeaiexamples_amd.training.full import FullTrainer, pretrain_batches
    from generativeaiexamples_amd.training.trainer import TrainConfig

    tok = small_byte_tokenizer(512)
    m = LlamaModel(LlamaConfig.tiny(num_layers=4), device=cuda, dist_ctx=DistContext()).random_init(1)
    texts = [synthetic.chunk_document(i, 120).page_content for i in range(200)]
    tr = FullTrainer(m, tok, TrainConfig(steps=30, global_batch=8, micro_batch=8, seq_len=128, lr=2e-3, warmup=3),
                     pretrain_batches(texts, tok, 128, 8))
    h = tr.train()
    assert h[-1] < h[0] - 1.0, h
    assert all(p.dtype == torch.bfloat16 for p in tr.params) and all(mm.dtype == torch.float32 for mm in tr.master)


def test_lora_on_served_fragment_layout_model(cuda):
    """a model an engine has served (projections rewritten in place into the fragment-ordered layout)
    LoRA-trains on its row-major values and merges correctly - same loss as an unconverted twin, and the merged,
    exported checkpoint equals the merge done on the twin."""
    from generativeaiexamples_amd import ops
    from generativeaiexamples_amd.training.forward import lm_loss
    from generativeaiexamples_amd.training.lora import LoRAAdapter

    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = LlamaConfig.tiny(hidden_size=512, intermediate_size=1024, num_heads=8, num_kv_heads=2, vocab_size=1024)
    served = LlamaModel(cfg, device="cuda", dist_ctx=ctx).random_init(seed=4)
    twin = LlamaModel(cfg, device="cuda", dist_ctx=ctx).random_init(seed=4)
    served.preshuffle_decode_weights(in_place=True)  # what LLMEngine does by default
    assert ops.is_frag(served.w["l0.qkv"]) and ops.is_frag(served.w["l1.down"])
    lcfg = LoRAConfig(r=8, alpha=16, targets=("qkv", "o", "gate_up", "down"))
    lora_s = LoRAAdapter(served, lcfg, device=cuda, seed=1)
    lora_t = LoRAAdapter(twin, lcfg, device=cuda, seed=1)
    with torch.no_grad():
        for k in lora_s.params:  # non-zero B so the adapters contribute
            lora_s.params[k].copy_(torch.randn_like(lora_s.params[k]) * 0.02)
            lora_t.params[k].copy_(lora_s.params[k])
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(3, 1000, (2, 64), generator=g).cuda()
    ls = lm_loss(served, lora_s, ids, ids.clone())
    lt = lm_loss(twin, lora_t, ids, ids.clone())
    assert torch.allclose(ls, lt, rtol=0, atol=1e-4), (ls.item(), lt.item())
    lora_s.merge_into(served)
    lora_t.merge_into(twin)
    assert ops.is_frag(served.w["l0.qkv"])
    a, b = served.export_hf_state(), twin.export_hf_state()
    for k in b:
        assert torch.equal(a[k], b[k]), k
