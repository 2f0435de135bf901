"""FM-radio streaming RAG (reference: /root/reference/community/fm-asr-streaming-rag): ``dsp`` (GPU signal chain),
``pipeline`` (packet receiver -> bursts -> PCM -> speech recogniser -> transcripts), ``stream_store`` (text
accumulator, timestamp database, vector retrieval), ``chains`` (intent-routed answers), ``server`` (chain server)."""
from .dsp import firwin, float_to_pcm16, fm_demod, lowpass, rational_factors, resample_poly  # noqa: F401
