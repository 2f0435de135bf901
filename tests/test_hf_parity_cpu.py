"""HF-checkpoint parity for the models the BASELINE configs run (VERDICT r3 "next" #7), against ``transformers``
on tiny random configs (no download): each reference model is written with ``save_pretrained`` and loaded back
through OUR checkpoint path (``models.registry`` from a HF directory), then compared on fp32 logits / features
and, for the generators, on engine greedy decoding (paged KV, chunked prefill, continuous batching).

* Llama-3 with ``rope_type: llama3`` frequency scaling (config 2's generator, docker-compose-nim-ms.yaml:4)
* Mixtral (config 5's agent model, query_decomposition_rag/chains.py:221-274)
* CLIP image and text towers (config 4's NV-CLIP search)
* Mllama (config 4's Llama-3.2-Vision, the NeVA replacement of custom_pdf_parser.py:52-78)
* the Mistral-based bidirectional reranker (docker-compose-nim-ms.yaml:60)
"""
import pytest
import torch

from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams

transformers = pytest.importorskip("transformers")


def _bf16_params(model, seed=0, norm_center=1.0):
    """Random weights that bf16 represents exactly (our models store bf16), norms around ``norm_center``."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if "norm" in n and n.endswith("weight") or "layernorm" in n and n.endswith("weight"):
                v = norm_center + 0.1 * torch.randn(p.shape, generator=g)
            elif n.endswith("gate") or "_gate" in n:
                v = 0.5 + 0.5 * torch.rand(p.shape, generator=g)  # tanh gates of Mllama: well away from 0
            else:
                v = 0.05 * torch.randn(p.shape, generator=g)
            p.copy_(v.to(torch.bfloat16).float())
    return model.float().eval()


def _feat(out):  # transformers 5 returns a model output (projected features in pooler_output), 4 a tensor
    return out if torch.is_tensor(out) else out.pooler_output


def _close(ours, ref, rel, what):
    err = (ours.float() - ref.float()).abs().max().item()
    assert err <= rel * ref.float().abs().max().item(), (what, err, ref.abs().max().item())


def _greedy_consistent(eng_out_ids, prompt, hf, rel=0.02, hf_kw=None):
    """Every engine-chosen token is the HF argmax at its prefix, up to a near-tie of ``rel`` of the logit scale."""
    ids = list(prompt)
    for t in eng_out_ids:
        with torch.no_grad():
            lg = hf(torch.tensor([ids]), **(hf_kw or {})).logits[0, -1].float()
        assert lg[t] >= lg.max() - rel * max(1.0, float(lg.abs().max())), (len(ids), t, int(lg.argmax()))
        ids.append(t)


def _engine(model, vocab):
    from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
    return LLMEngine(model, small_byte_tokenizer(vocab), EngineConfig(
        max_num_seqs=4, max_batched_tokens=64, prefill_chunk=24, num_blocks=96, max_model_len=512, use_graphs=False))


# ---------------------------------------------------------------------------------------------- Llama-3 (llama3 rope)
def test_llama3_rope_scaling_matches_transformers(tmp_path):
    from generativeaiexamples_amd.models.registry import build_llm
    # original_max_position_embeddings 64 puts head_dim 64's frequencies in all three llama3 regimes
    # (kept, smoothly interpolated, divided by the factor) on a tiny model
    rs = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
          "original_max_position_embeddings": 64}
    hf = transformers.LlamaForCausalLM(transformers.LlamaConfig(
        vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, max_position_embeddings=1024, rope_scaling=rs, rope_theta=500000.0, rms_norm_eps=1e-5,
        bos_token_id=1, eos_token_id=2, tie_word_embeddings=False))
    hf = _bf16_params(hf)
    hf.save_pretrained(tmp_path)
    m, _, _ = build_llm(weights=str(tmp_path), device="cpu")
    assert m.cfg.rope_scaling and m.cfg.rope_scaling["factor"] == 8.0 and m.cfg.rope_theta == 500000.0
    ids = torch.randint(3, 500, (150,), generator=torch.Generator().manual_seed(1))  # past 64: scaled regime
    with torch.no_grad():
        ref = hf(ids[None]).logits[0]
    _close(m.reference_forward(ids), ref, 1e-3, "llama3 logits")
    prompt = ids[:97].tolist()
    r = _engine(m, 512).generate([prompt], SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))[0]
    assert len(r.output_ids) == 6
    _greedy_consistent(r.output_ids, prompt, hf)


# ---------------------------------------------------------------------------------------------- Mixtral
def test_mixtral_matches_transformers(tmp_path):
    from generativeaiexamples_amd.models.mixtral import MixtralModel
    from generativeaiexamples_amd.models.registry import build_llm
    hf = transformers.MixtralForCausalLM(transformers.MixtralConfig(
        vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
        num_key_value_heads=2, num_local_experts=4, num_experts_per_tok=2, max_position_embeddings=1024,
        rope_theta=1e6, bos_token_id=1, eos_token_id=2, tie_word_embeddings=False))
    hf = _bf16_params(hf, seed=3)
    # the router logits are tiny at 0.05-scale weights; widen them so the top-2 choice is not a coin flip
    with torch.no_grad():
        for layer in hf.model.layers:
            layer.mlp.gate.weight.mul_(8.0)
    hf.save_pretrained(tmp_path)  # on-disk names: block_sparse_moe.experts.{e}.w{1,2,3}
    m, _, _ = build_llm(weights=str(tmp_path), device="cpu")
    assert isinstance(m, MixtralModel) and m.cfg.num_experts == 4 and m.cfg.top_k == 2
    ids = torch.randint(3, 500, (40,), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        ref = hf(ids[None]).logits[0]
    _close(m.reference_forward(ids), ref, 1e-3, "mixtral logits")
    prompt = ids[:33].tolist()
    r = _engine(m, 512).generate([prompt], SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))[0]
    assert len(r.output_ids) == 5
    _greedy_consistent(r.output_ids, prompt, hf)


# ---------------------------------------------------------------------------------------------- CLIP
def test_clip_features_match_transformers(tmp_path):
    from generativeaiexamples_amd.models.clip import ClipModel
    from generativeaiexamples_amd.models.registry import build_encoder
    hf = transformers.CLIPModel(transformers.CLIPConfig(
        text_config=dict(vocab_size=1024, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                         num_attention_heads=2, max_position_embeddings=77, eos_token_id=1023, bos_token_id=1022,
                         pad_token_id=1),
        vision_config=dict(hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=2,
                           image_size=56, patch_size=14),
        projection_dim=96))
    hf = _bf16_params(hf, seed=4)
    hf.save_pretrained(tmp_path)
    m, _, _ = build_encoder(weights=str(tmp_path), device="cpu")
    assert isinstance(m, ClipModel)
    px = torch.rand(3, 3, 56, 56, generator=torch.Generator().manual_seed(5))
    mean = torch.tensor([0.48145466, 0.4578275, 0.40821073]).view(1, 3, 1, 1)
    std = torch.tensor([0.26862954, 0.26130258, 0.27577711]).view(1, 3, 1, 1)
    with torch.no_grad():
        ref_i = torch.nn.functional.normalize(_feat(hf.get_image_features(pixel_values=(px - mean) / std)), dim=-1)
    _close(m.reference_encode_image(px), ref_i, 2e-3, "clip image (fp32 oracle)")
    assert torch.nn.functional.cosine_similarity(m.encode_image(px), ref_i).min() > 0.999
    toks = [[1022, 5, 17, 300, 1023], [1022, 900, 4, 8, 9, 10, 11, 1023]]  # EOT = the highest id, last
    e = m.encode_text(toks)
    for row, t in zip(e, toks):
        with torch.no_grad():
            ref_t = torch.nn.functional.normalize(_feat(hf.get_text_features(input_ids=torch.tensor([t]))), dim=-1)[0]
        assert torch.nn.functional.cosine_similarity(row[None], ref_t[None]).item() > 0.999


# ---------------------------------------------------------------------------------------------- Mistral reranker
def test_decoder_reranker_matches_bidirectional_mistral(tmp_path):
    """The NV-RerankQA-Mistral class: a Mistral decoder run with bidirectional attention over the pair, mean-pooled
    after the final norm, linear score. The HF side is MistralModel with an all-visible 4-D mask."""
    from generativeaiexamples_amd.models.decoder_reranker import DecoderRerankerModel
    from generativeaiexamples_amd.models.registry import build_reranker_service
    cfg = transformers.MistralConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                     num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024,
                                     rope_theta=1e6, sliding_window=None, bos_token_id=1, eos_token_id=2)
    hf = transformers.MistralForSequenceClassification(cfg.__class__(**{**cfg.to_dict(), "num_labels": 1}))
    hf = _bf16_params(hf, seed=6)
    hf.save_pretrained(tmp_path)
    svc, _ = build_reranker_service(weights=str(tmp_path), device="cpu")
    m = svc.model
    assert isinstance(m, DecoderRerankerModel) and m.cfg.num_layers == 2 and m.cfg.hidden_size == 256
    g = torch.Generator().manual_seed(7)
    lens = [13, 30, 21]
    ids = torch.randint(3, 500, (sum(lens),), generator=g)
    ref, o = [], 0
    for n in lens:
        t = ids[o:o + n][None]
        o += n
        with torch.no_grad():
            h = hf.model(input_ids=t, attention_mask=torch.zeros(1, 1, n, n)).last_hidden_state[0]  # after final norm
        ref.append(h.mean(0) @ hf.score.weight[0])
    ref = torch.stack(ref)
    _close(m.reference_score(ids, lens), ref, 1e-3, "reranker oracle")
    cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32)
    _close(m.score(ids.int(), cu, lens), ref, 3e-2, "reranker engine path")


# ---------------------------------------------------------------------------------------------- Mllama
_TF5 = int(transformers.__version__.split(".")[0]) >= 5
OURS_INTER = (1, 2)  # two kept layers: their channel interleave in the projector input is pinned too
HF_INTER = [i - 1 for i in OURS_INTER] if _TF5 else list(OURS_INTER)

def test_mllama_matches_transformers(tmp_path):
    """Text-only and image+text logits of Llama-3.2-Vision's architecture (tiles padded to a multiple of 8 tokens,
    absent tiles, the tile attention mask, gated positional embeddings, global layers, interleaved intermediate
    features, gated cross-attention layers) against MllamaForConditionalGeneration, image token first.

    Text rows BEFORE the image token follow Meta's reference (no cross-attention and no cross-MLP contribution);
    transformers lets such rows attend every tile unmasked and zeroes only their MLP term, so mid-prompt images
    are pinned by an invariant instead: those rows equal the text-only forward."""
    from generativeaiexamples_amd.models.mllama import ImageInput, MllamaModel
    from generativeaiexamples_amd.models.registry import build_llm
    V, T_img = 512, 500
    hf = transformers.MllamaForConditionalGeneration(transformers.MllamaConfig(
        vision_config=dict(hidden_size=128, num_hidden_layers=3, num_global_layers=1, attention_heads=2,
                           intermediate_size=256, image_size=56, patch_size=14, max_num_tiles=4,
                           intermediate_layers_indices=HF_INTER, vision_output_dim=384, norm_eps=1e-5),
        text_config=dict(vocab_size=V, hidden_size=256, intermediate_size=512, num_hidden_layers=4,
                         num_attention_heads=4, num_key_value_heads=2, cross_attention_layers=[1, 3],
                         max_position_embeddings=1024, rope_theta=500000.0, rms_norm_eps=1e-5, bos_token_id=1,
                         eos_token_id=2, pad_token_id=3),
        image_token_index=V))
    hf = _bf16_params(hf, seed=8)
    with torch.no_grad():  # HF inits gates at 0; make every gated path live (tanh(gate) well away from 0 and 1)
        for n, p in hf.named_parameters():
            if n.split(".")[-1] in ("gate_attn", "gate_ffn", "gate", "cross_attn_attn_gate", "cross_attn_mlp_gate"):
                p.copy_(torch.full_like(p, 0.75))
    hf.save_pretrained(tmp_path)
    m, _, _ = build_llm(weights=str(tmp_path), device="cpu")
    assert isinstance(m, MllamaModel)
    # Meta's encoder (and transformers 4) keeps the hidden state ENTERING layer i for index i; transformers 5
    # collects the state LEAVING layer i, one layer later. Ours follows Meta: pin the same tensors.
    m.mcfg.vision.intermediate_layers = OURS_INTER
    g = torch.Generator().manual_seed(9)
    ids = torch.randint(3, 500, (40,), generator=g)
    ids[0] = V  # <|image|>
    with torch.no_grad():  # text only: cross layers skipped on both sides
        ref = hf(input_ids=ids[None]).logits[0]
    _close(m.reference_forward(ids), ref, 1e-3, "mllama text-only")
    # a 2x1 tile canvas (aspect ratio id 2 of 4 tiles: (w, h) = (1, 2))
    ntiles, ar = 2, 2
    px = torch.rand(ntiles, 3, 56, 56, generator=g)
    mean = torch.tensor([0.48145466, 0.4578275, 0.40821073]).view(1, 3, 1, 1)
    std = torch.tensor([0.26862954, 0.26130258, 0.27577711]).view(1, 3, 1, 1)
    pv = torch.zeros(1, 1, 4, 3, 56, 56)
    pv[0, 0, :ntiles] = (px - mean) / std
    ar_mask = torch.zeros(1, 1, 4, dtype=torch.long)
    ar_mask[0, 0, :ntiles] = 1
    xmask = torch.zeros(1, ids.numel(), 1, 4, dtype=torch.long)
    xmask[0, :, 0, :ntiles] = 1  # the processor's mask: tokens from the image token on see its tiles
    with torch.no_grad():
        ref = hf(input_ids=ids[None], pixel_values=pv, aspect_ratio_ids=torch.tensor([[ar]]),
                 aspect_ratio_mask=ar_mask, cross_attention_mask=xmask).logits[0]
    im = ImageInput(px, ar, ntiles)
    _close(m.reference_forward(ids, im), ref, 2e-3, "mllama image+text")
    # the engine path (paged cross cache, row masks, chunked prefill) agrees with HF's greedy choice
    prompt = ids[:30].tolist()
    eng = _engine(m, 520)
    r = eng.add_request(prompt, SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True), images=[im])
    while eng.has_work():
        eng.step()
    assert len(r.output_ids) == 4
    L = len(prompt)
    xm = torch.zeros(1, L + 4, 1, 4, dtype=torch.long)
    xm[0, :, 0, :ntiles] = 1
    ids_all = list(prompt)
    for t in r.output_ids:
        with torch.no_grad():
            n = len(ids_all)
            lg = hf(input_ids=torch.tensor([ids_all]), pixel_values=pv, aspect_ratio_ids=torch.tensor([[ar]]),
                    aspect_ratio_mask=ar_mask, cross_attention_mask=xm[:, :n]).logits[0, -1]
        assert lg[t] >= lg.max() - 0.02 * max(1.0, float(lg.abs().max())), (n, t, int(lg.argmax()))
        ids_all.append(t)

    # mid-prompt image: rows before the token are exactly the text-only forward, rows after it see the image
    ids2 = ids.clone()
    ids2[0], ids2[9] = 7, V
    text_only, with_img = m.reference_forward(ids2), m.reference_forward(ids2, im)
    assert torch.equal(with_img[:9], text_only[:9])
    assert (with_img[9:] - text_only[9:]).abs().max() > 1e-2
    eng = _engine(m, 520)
    req = eng.add_request(ids2.tolist(), SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True), images=[im])
    while eng.has_work():
        eng.step()
    lg = with_img[-1]
    assert lg[req.output_ids[0]] >= lg.max() - 0.02 * max(1.0, float(lg.abs().max()))
