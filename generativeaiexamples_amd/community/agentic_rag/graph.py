"""A small state-graph runner for agentic RAG flows (the LangGraph ``StateGraph`` role in
/root/reference/community/log_analysis_multi_agent_rag/bat_ai.py:29-61: nodes that return state updates, plain edges,
conditional edges routed by a function of the state, START / END).

Nodes run in the calling thread; a node that fans out (e.g. grading every retrieved document) does its own concurrency
so the in-process LLM engine batches the calls. ``max_steps`` bounds every run, so a flow whose conditional edges loop
(rewrite -> retrieve -> grade -> rewrite ...) always ends. ``trace`` records the visited nodes.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

START, END = "__start__", "__end__"

Node = Callable[[dict], Optional[dict]]


class GraphRecursionError(RuntimeError):
    pass


class StateGraph:
    def __init__(self):
        self.nodes: Dict[str, Node] = {}
        self.edges: Dict[str, str] = {}
        self.cond: Dict[str, Tuple[Callable[[dict], str], Dict[str, str]]] = {}

    def add_node(self, name: str, fn: Node) -> "StateGraph":
        if name in (START, END) or name in self.nodes:
            raise ValueError(f"bad or duplicate node name {name!r}")
        self.nodes[name] = fn
        return self

    def add_edge(self, src: str, dst: str) -> "StateGraph":
        if src in self.edges or src in self.cond:
            raise ValueError(f"node {src!r} already has an outgoing edge")
        self.edges[src] = dst
        return self

    def add_conditional_edges(self, src: str, router: Callable[[dict], str], mapping: Dict[str, str]) -> "StateGraph":
        if src in self.edges or src in self.cond:
            raise ValueError(f"node {src!r} already has an outgoing edge")
        self.cond[src] = (router, dict(mapping))
        return self

    def compile(self, max_steps: int = 25) -> "CompiledGraph":
        for src, dst in list(self.edges.items()):
            for n in (src, dst):
                if n not in self.nodes and n not in (START, END):
                    raise ValueError(f"edge references unknown node {n!r}")
        for src, (_, mapping) in self.cond.items():
            for n in [src, *mapping.values()]:
                if n not in self.nodes and n not in (START, END):
                    raise ValueError(f"conditional edge references unknown node {n!r}")
        if START not in self.edges and START not in self.cond:
            raise ValueError("the graph needs an edge from START")
        return CompiledGraph(self, max_steps)


class CompiledGraph:
    def __init__(self, g: StateGraph, max_steps: int):
        self.g, self.max_steps = g, max_steps

    def _next(self, cur: str, state: dict) -> str:
        if cur in self.g.cond:
            router, mapping = self.g.cond[cur]
            key = router(state)
            if key not in mapping:
                raise KeyError(f"router of {cur!r} returned {key!r}, not one of {sorted(mapping)}")
            return mapping[key]
        if cur in self.g.edges:
            return self.g.edges[cur]
        return END

    def invoke(self, state: dict) -> dict:
        state = dict(state)
        trace: List[str] = []
        cur = self._next(START, state)
        for _ in range(self.max_steps):
            if cur == END:
                state["trace"] = trace
                return state
            update = self.g.nodes[cur](state) or {}
            state.update(update)
            trace.append(cur)
            cur = self._next(cur, state)
        if cur == END:
            state["trace"] = trace
            return state
        raise GraphRecursionError(f"no END after {self.max_steps} steps: {' -> '.join(trace[-8:])}")
