"""Community projects of the reference re-built on this framework: the FM-radio streaming RAG app
(``fm_asr``: SDR signal chain on HIP kernels, transcript accumulator, time-aware retrieval, chain server) and the
digital-fingerprinting autoencoder (``dfp``)."""
