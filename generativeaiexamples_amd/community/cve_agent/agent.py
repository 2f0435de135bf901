"""Tool-using agent that answers one checklist item about a container (reference: /root/reference/community/
event-driven-rag-cve-analysis/cyber_dev_day/pipeline_utils.py:43-112 - a LangChain zero-shot ReAct agent with the
SBOM and code-QA tools, a system prompt that restricts it to the checklist item and a retry message for malformed
steps).

The loop is the text ReAct protocol, so any chat model drives it: the model writes ``Thought`` / ``Action`` /
``Action Input`` (generation stops before ``Observation:``), the tool runs, its output is appended as the observation,
until the model writes ``Final Answer``. A step with neither is answered with a format reminder (up to
``max_parse_errors``) and the loop ends after ``max_steps`` with the last thought as the answer.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from .tools import Tool

AGENT_SYSTEM = (
    "You investigate a container image for one checklist item about a vulnerability. Answer only that item; do not "
    "investigate anything else. Facts about the container are available only through the tools below.\n\n"
    "Tools:\n{tools}\n\n"
    "Work in steps. Each reply is either\n"
    "Thought: <reasoning>\nAction: <one of [{names}]>\nAction Input: <the exact input, nothing after it>\n"
    "(then wait for the Observation), or\n"
    "Thought: <reasoning>\nFinal Answer: <the answer to the checklist item, with the evidence you found>\n"
    "Never write an Observation yourself and never give an Action and a Final Answer in the same reply.")
FORMAT_REMINDER = ("Your reply did not follow the format. Reply with 'Thought:' and then either 'Action:' + "
                   "'Action Input:' or 'Final Answer:'.")

_FINAL = re.compile(r"Final Answer\s*:\s*(.*)", re.S | re.I)
_ACTION = re.compile(r"Action\s*:\s*(.*?)\s*\n+\s*Action Input\s*:\s*(.*?)\s*(?:\n|$)", re.S | re.I)


@dataclass
class AgentResult:
    answer: str
    steps: List[Tuple[str, str, str]] = field(default_factory=list)  # (action, input, observation)
    finished: bool = True


def parse_step(text: str) -> Tuple[Optional[str], Optional[str], Optional[str]]:
    """(final answer, action, action input); the earliest of an action / a final answer wins."""
    fa, ac = _FINAL.search(text), _ACTION.search(text)
    if fa and (not ac or fa.start() < ac.start()):
        return fa.group(1).strip(), None, None
    if ac:
        arg = ac.group(2).strip().strip("`").strip()
        if len(arg) >= 2 and arg[0] == arg[-1] and arg[0] in "'\"":
            arg = arg[1:-1]
        return None, ac.group(1).strip().strip("[]`*"), arg
    return None, None, None


class ReActAgent:
    def __init__(self, llm, tools: Sequence[Tool], max_steps: int = 8, max_parse_errors: int = 2,
                 max_tokens: int = 384):
        self.llm, self.tools = llm, {t.name.lower(): t for t in tools}
        self.max_steps, self.max_parse_errors, self.max_tokens = max_steps, max_parse_errors, max_tokens
        self.system = AGENT_SYSTEM.format(tools="\n".join(f"- {t.name}: {t.description}" for t in tools),
                                          names=", ".join(t.name for t in tools))

    def _tool(self, name: str) -> Optional[Tool]:
        key = name.lower()
        return self.tools.get(key) or next((t for k, t in self.tools.items() if key in k or k in key), None)

    def run(self, question: str) -> AgentResult:
        transcript, steps, errors, last = "", [], 0, ""
        for _ in range(self.max_steps):
            reply = self.llm.invoke([{"role": "system", "content": self.system},
                                     {"role": "user", "content": f"Checklist item: {question}\n{transcript}"}],
                                    temperature=0.0, max_tokens=self.max_tokens, stop=["\nObservation:"])
            reply = getattr(reply, "content", reply) or ""
            final, action, arg = parse_step(reply)
            if final is not None:
                return AgentResult(final, steps)
            if action is None:
                errors += 1
                last = reply.strip() or last
                if errors > self.max_parse_errors:
                    break
                transcript += f"{reply.strip()}\n{FORMAT_REMINDER}\n"
                continue
            tool = self._tool(action)
            obs = tool(arg) if tool is not None else \
                f"'{action}' is not a tool. Use one of: {', '.join(t.name for t in self.tools.values())}."
            steps.append((action, arg, obs))
            head = reply[: _ACTION.search(reply).end()].strip()
            transcript += f"{head}\nObservation: {obs}\n"
            last = obs
        m = re.findall(r"Thought\s*:\s*(.*)", transcript)
        return AgentResult(m[-1].strip() if m else last, steps, finished=False)
