"""Parallelism over RCCL/xGMI (one process per GPU, ``torch.distributed`` backend ``nccl`` = RCCL).

* :mod:`.dist`  - process-group setup (env:// rendezvous), TP / DP / EP sub-groups, collectives
  with a gloo fallback for the CPU test tier.
* :mod:`.tp`    - tensor-parallel sharding rules for column / row parallel linears and the
  vocab-parallel embedding / LM head.
* :mod:`.ep`    - expert-parallel all-to-all dispatch/combine for MoE.
"""
from .dist import DistContext, get_context, init_distributed  # noqa: F401
