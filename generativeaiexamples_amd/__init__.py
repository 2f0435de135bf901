"""generativeaiexamples_amd - an MI355X-native (gfx950) RAG serving framework.

Same capabilities and API surface as NVIDIA GenerativeAIExamples' RAG stack
(chain-server REST API, NIM/OpenAI-compatible ``/v1`` endpoints, example
pipelines, playground, evaluation and observability tools), rebuilt around one
PyTorch-ROCm engine: hand-written CDNA4 HIP kernels (``csrc/kernels``), a C++
host runtime (``csrc/runtime``), RCCL-over-xGMI parallelism (``parallel``) and
an exact HBM-resident vector index (``index``).
"""
__version__ = "0.1.0"
