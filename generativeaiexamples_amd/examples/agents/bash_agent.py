"""Tool-calling bash agent over the OpenAI-compatible /v1 API (reference
nemotron/LLM/bash_computer_use_agent: an OpenAI tool-call loop with an allow-listed shell tool,
plus W12's "detailed thinking on/off" system-prompt switch).

The model is offered one tool, ``exec_bash_command(cmd)``. Each turn: POST the conversation + tool
schema to /v1/chat/completions; when the reply carries ``tool_calls`` the command is checked against
the allow-list (first word) and parsed option by option against a per-command option ALLOW-list
(short clusters, attached values such as ``-n5``, exact long options only - GNU's abbreviated long
options never match; ``find`` predicates from their own table). Every path operand and every path-valued
option must resolve inside the working directory. The command is then optionally confirmed by the user,
run in that directory with a timeout, and its stdout/stderr returned as a ``tool`` message; a reply
without tool calls ends the loop.

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

class _Spec:
    """Allowed options of one command: short flags without / with a value, exact long options without / with a
    value (``--opt=value`` or ``--opt value``), which option values are paths, and the positional limit."""

    def __init__(self, flags: str = "", valued: str = "", longs=(), long_valued=(), path_opts=(), max_pos: int = 64):
        self.flags, self.valued = set(flags), set(valued)
        self.longs, self.long_valued, self.path_opts, self.max_pos = set(longs), set(long_valued), set(path_opts), max_pos


_SPECS = {
    "ls": _Spec("alhRtrSs1dFi", longs=("--all", "--human-readable", "--recursive", "--reverse")),
    "cat": _Spec("nbsAET", longs=("--number",)),
    "head": _Spec("qv", "nc", long_valued=("--lines", "--bytes")),
    "tail": _Spec("qv", "nc", long_valued=("--lines", "--bytes")),  # no -f: it never returns
    "wc": _Spec("lwcmL", longs=("--lines", "--words", "--bytes", "--chars")),
    "grep": _Spec("ivnclLwxohHEFsq", "emABC", longs=("--ignore-case", "--count", "--line-number"),
                  long_valued=("--regexp", "--max-count", "--include", "--exclude")),
    "pwd": _Spec(max_pos=0),
    "echo": _Spec("ne"),
    "sort": _Spec("rnufhVbsM", "kt", longs=("--reverse", "--numeric-sort", "--unique"), long_valued=("--key",)),
    "uniq": _Spec("cdui", max_pos=1),  # a second operand would be an OUTPUT file
    "du": _Spec("shac", "d", longs=("--summarize", "--human-readable"), long_valued=("--max-depth",)),
    "df": _Spec("hT", longs=("--human-readable",)),
    "date": _Spec("uIR"),
}
# find predicates -> number of values; values of the path-valued ones are path-checked. Anything that executes,
# deletes, writes or follows symlinks (-exec, -ok, -delete, -fprint*, -fls, -L, -follow) is simply absent.
_FIND_PREDS = {"-name": 1, "-iname": 1, "-path": 1, "-ipath": 1, "-regex": 1, "-type": 1, "-maxdepth": 1,
               "-mindepth": 1, "-size": 1, "-mtime": 1, "-mmin": 1, "-newer": 1, "-empty": 0, "-print": 0,
               "-not": 0, "!": 0, "-o": 0, "-a": 0, "-or": 0, "-and": 0, "(": 0, ")": 0}
_FIND_PATH_VALUES = {"-newer"}


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

    def _check_args(self, argv: List[str]) -> Optional[str]:
        """None when every option is allowed for this command and every path stays inside the working directory."""
        cmd, args = argv[0], argv[1:]
        paths: List[str] = []
        if cmd == "find":
            i = 0
            while i < len(args) and not (args[i].startswith("-") or args[i] in ("!", "(", ")")):
                paths.append(args[i])  # starting points
                i += 1
            while i < len(args):
                a = args[i]
                if a not in _FIND_PREDS:
                    return f"error: find predicate {a!r} is not allowed"
                n = _FIND_PREDS[a]
                if i + n >= len(args) + (0 if n else 1):
                    return f"error: find predicate {a} needs a value"
                if a in _FIND_PATH_VALUES:
                    paths.append(args[i + 1])
                i += 1 + n
        else:
            spec = _SPECS.get(cmd)
            if spec is None:
                return f"error: '{cmd}' is not allowed"
            pos: List[str] = []
            i, end_of_opts = 0, False
            while i < len(args):
                a = args[i]
                i += 1
                if end_of_opts or a == "-" or not a.startswith("-"):
                    pos.append(a)
                elif a == "--":
                    end_of_opts = True
                elif a.startswith("--"):
                    name, eq, val = a.partition("=")
                    if name in spec.longs and not eq:
                        continue
                    if name not in spec.long_valued:  # exact names only: no GNU abbreviations
                        return f"error: option {name} is not allowed for {cmd}"
                    if not eq:
                        if i >= len(args):
                            return f"error: option {name} needs a value"
                        val = args[i]
                        i += 1
                    if name in spec.path_opts:
                        paths.append(val)
                else:  # short cluster, e.g. -la or -n5 / -n 5
                    for j, ch in enumerate(a[1:], 1):
                        if ch in spec.flags:
                            continue
                        if ch not in spec.valued:
                            return f"error: option -{ch} is not allowed for {cmd}"
                        if j + 1 == len(a):  # value is the next argument
                            if i >= len(args):
                                return f"error: option -{ch} needs a value"
                            i += 1
                        break  # the rest of the cluster is the attached value
            if len(pos) > spec.max_pos:
                return f"error: too many operands for {cmd}"
            paths += pos
        for p in paths:
            if not self._inside(p):
                return f"error: path {p!r} is outside the working directory"
        return None

    def __call__(self, cmd: str) -> str:
        try:
            argv = shlex.split(cmd)
        except ValueError as e:
            return f"error: cannot parse command ({e})"
        if not argv or argv[0] not in self.allowed:
            return f"error: '{argv[0] if argv else ''}' is not allowed; allowed: {', '.join(sorted(self.allowed))}"
        if any(tok in cmd for tok in (";", "&&", "||", "|", "`", "$(", ">", "<", "\n")):
            return "error: command chaining, pipes and redirection are not allowed"
        err = self._check_args(argv)
        if err:
            return err
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
