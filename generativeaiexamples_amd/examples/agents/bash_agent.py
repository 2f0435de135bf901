"""Tool-calling bash agent over the OpenAI-compatible /v1 API (reference
nemotron/LLM/bash_computer_use_agent: an OpenAI tool-call loop with an allow-listed shell tool,
plus W12's "detailed thinking on/off" system-prompt switch).

The model is offered one tool, ``exec_bash_command(cmd)``. Each turn: POST the conversation + tool
schema to /v1/chat/completions; when the reply carries ``tool_calls`` the command is checked against
the allow-list (first word), its flags (no ``find -exec/-delete/...``) and its path arguments (each must
resolve inside the working directory), optionally confirmed by the user, run in that directory with a
timeout, and its stdout/stderr returned as a ``tool`` message; a reply without tool calls
ends the loop.

    python -m generativeaiexamples_amd.examples.agents.bash_agent --base-url http://localhost:8000 \\
        --model meta/llama3-8b-instruct --cwd /tmp/sandbox "How many .txt files are here?"
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
from typing import Callable, List, Optional

ALLOWED = ("ls", "cat", "head", "tail", "wc", "grep", "find", "pwd", "echo", "sort", "uniq", "du", "df", "date")
# options that execute, delete or write files (find), or follow arbitrary paths outside the sandbox
_BANNED_FLAGS = {"find": {"-exec", "-execdir", "-ok", "-okdir", "-delete", "-fprint", "-fprint0", "-fprintf", "-fls",
                          "-L", "-follow"},
                 "grep": {"-r", "-R", "--dereference-recursive"},
                 "sort": {"-o", "--output", "-T", "--temporary-directory", "--compress-program"}}
_BANNED_FLAG_PREFIXES = {"sort": ("--output=", "--temporary-directory=", "--compress-program="),
                         "grep": ("--dereference",)}
TOOL = {"type": "function", "function": {
    "name": "exec_bash_command", "description": "Execute an allow-listed bash command and return its output.",
    "parameters": {"type": "object", "properties": {"cmd": {"type": "string", "description": "the command"}},
                   "required": ["cmd"]}}}


class BashTool:
    def __init__(self, cwd: str, allowed=ALLOWED, timeout: float = 10.0, confirm: Optional[Callable[[str], bool]] = None):
        self.cwd, self.allowed, self.timeout, self.confirm = os.path.realpath(cwd), set(allowed), timeout, confirm

    def _inside(self, arg: str) -> bool:
        """True when ``arg``, read as a path relative to the working directory (``~`` expanded, symlinks
        resolved), stays inside it. Non-path arguments (patterns, numbers) resolve inside trivially."""
        p = os.path.realpath(os.path.join(self.cwd, os.path.expanduser(arg)))
        return p == self.cwd or p.startswith(self.cwd + os.sep)

    def __call__(self, cmd: str) -> str:
        try:
            argv = shlex.split(cmd)
        except ValueError as e:
            return f"error: cannot parse command ({e})"
        if not argv or argv[0] not in self.allowed:
            return f"error: '{argv[0] if argv else ''}' is not allowed; allowed: {', '.join(sorted(self.allowed))}"
        if any(tok in cmd for tok in (";", "&&", "||", "|", "`", "$(", ">", "<", "\n")):
            return "error: command chaining, pipes and redirection are not allowed"
        bad = [a for a in argv[1:] if a in _BANNED_FLAGS.get(argv[0], ()) or
               any(a.startswith(p) for p in _BANNED_FLAG_PREFIXES.get(argv[0], ()))]
        if bad:
            return f"error: option {bad[0]} is not allowed for {argv[0]}"
        for a in argv[1:]:
            if a.startswith("-") and "=" not in a:
                continue
            path = a.split("=", 1)[1] if a.startswith("-") else a
            if not self._inside(path):
                return f"error: path {path!r} is outside the working directory"
        if self.confirm is not None and not self.confirm(cmd):
            return "error: the user declined to run this command"
        try:
            r = subprocess.run(argv, cwd=self.cwd, capture_output=True, text=True, timeout=self.timeout)
        except subprocess.TimeoutExpired:
            return f"error: timed out after {self.timeout}s"
        out = (r.stdout + (("\nstderr: " + r.stderr) if r.stderr else "")).strip()
        return out[:8000] if out else f"(exit code {r.returncode}, no output)"


def system_prompt(cwd: str, thinking: Optional[str]) -> str:
    s = (f"You are a helpful assistant operating a Linux shell in the directory {cwd}. Use the exec_bash_command "
         "tool to inspect files when needed, then answer the user concisely.")
    if thinking in ("on", "off"):
        s = f"detailed thinking {thinking}\n\n" + s
    return s


def run_agent(question: str, chat: Callable[[List[dict], List[dict]], dict], tool: BashTool, max_turns: int = 8,
              thinking: Optional[str] = None) -> str:
    """chat(messages, tools) -> assistant message dict (OpenAI format)."""
    msgs = [{"role": "system", "content": system_prompt(tool.cwd, thinking)}, {"role": "user", "content": question}]
    for _ in range(max_turns):
        msg = chat(msgs, [TOOL])
        calls = msg.get("tool_calls") or []
        msgs.append({"role": "assistant", "content": msg.get("content"), **({"tool_calls": calls} if calls else {})})
        if not calls:
            return msg.get("content") or ""
        for c in calls:
            try:
                args = json.loads(c["function"].get("arguments") or "{}")
            except json.JSONDecodeError:
                args = {}
            out = tool(args.get("cmd", "")) if c["function"]["name"] == "exec_bash_command" else "error: unknown tool"
            msgs.append({"role": "tool", "tool_call_id": c.get("id", ""), "content": out})
    return "stopped: too many tool calls"


def http_chat(base_url: str, model: str, temperature: float = 0.2, max_tokens: int = 512):
    import httpx
    url = base_url.rstrip("/") + "/v1/chat/completions"

    def chat(messages, tools):
        r = httpx.post(url, json={"model": model, "messages": messages, "tools": tools, "tool_choice": "auto",
                                  "temperature": temperature, "max_tokens": max_tokens}, timeout=600)
        r.raise_for_status()
        return r.json()["choices"][0]["message"]
    return chat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("question")
    ap.add_argument("--base-url", default="http://localhost:8000")
    ap.add_argument("--model", default="meta/llama3-8b-instruct")
    ap.add_argument("--cwd", default=".")
    ap.add_argument("--thinking", choices=["on", "off"], default=None)
    ap.add_argument("--yes", action="store_true", help="run allowed commands without asking")
    a = ap.parse_args()
    confirm = None if a.yes else (lambda cmd: input(f"run `{cmd}`? [y/N] ").strip().lower() == "y")
    print(run_agent(a.question, http_chat(a.base_url, a.model), BashTool(a.cwd, confirm=confirm), thinking=a.thinking))


if __name__ == "__main__":
    main()
