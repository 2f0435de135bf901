"""PandasAI LLM adapter (reference RAG/src/pandasai/llms/nv_aiplay.py:31-106, an ``LLM``
subclass whose ``call(instruction, context)`` renders the PandasAI prompt and sends it to ChatNVIDIA).

``MI355XPandasLLM`` keeps that duck-typed surface (``type``, ``call``, ``last_prompt``, the
``temperature`` / ``top_p`` / ``max_tokens`` / ``model`` params) and routes the prompt to the
configured chain-server LLM: in-process engine (``APP_LLM_MODELENGINE=mi355x``) or any
NIM/OpenAI-compatible ``/v1`` server. pandasai itself is optional - when it is importable the adapter
also registers as a subclass of its ``LLM`` base so ``SmartDataframe(df, config={"llm": ...})`` accepts
it; the structured-data example uses the framework's own sandboxed pandas evaluator either way.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

try:  # pragma: no cover - pandasai is not part of this image
    from pandasai.llm.base import LLM as _Base
except Exception:  # noqa: BLE001
    _Base = object


class MI355XPandasLLM(_Base):
    def __init__(self, model: Optional[str] = None, temperature: float = 0.1, top_p: float = 1.0,
                 max_tokens: int = 1000, llm=None):
        from ..chain_server.utils import get_config
        self.model = model or get_config().llm.model_name_pandas_ai or get_config().llm.model_name
        self.temperature, self.top_p, self.max_tokens = temperature, top_p, max_tokens
        self._llm = llm
        self.last_prompt = ""

    @property
    def type(self) -> str:
        return "mi355x-llm"

    @property
    def _default_params(self) -> Dict[str, Any]:
        return {"model": self.model, "temperature": self.temperature, "top_p": self.top_p,
                "max_tokens": self.max_tokens}

    def _chat(self):
        if self._llm is None:
            from ..chain_server.utils import get_llm
            self._llm = get_llm(temperature=self.temperature, top_p=self.top_p, max_tokens=self.max_tokens)
        return self._llm

    def call(self, instruction: Any, context: Any = None, suffix: str = "") -> str:
        prompt = instruction.to_string() if hasattr(instruction, "to_string") else str(instruction)
        self.last_prompt = prompt + suffix
        return self._chat().invoke([{"role": "user", "content": self.last_prompt}])
