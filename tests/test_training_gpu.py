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
