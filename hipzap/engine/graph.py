"""Model-agnostic lowered IR + static memory planner.

A model lowers itself (``models/*.py: build_graph``) into a :class:`Graph`: a topologically
ordered list of kernel nodes over symbolic tensors with static shapes. The planner assigns
every internal tensor an offset in ONE activation arena, reusing memory between tensors
whose lifetimes do not overlap (greedy best-fit by size, the classic static-allocation
scheme). Side-stream branches (``fork``/``join``) extend the lifetime of everything they
touch to the whole fork..join window, so concurrent branches never alias.
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field

import torch

ALIGN = 256


@dataclass
class TensorSpec:
    shape: tuple
    dtype: torch.dtype
    name: str
    external: bool = False  # graph input/output: owned by the context, not the arena

    @property
    def nbytes(self) -> int:
        n = 1
        for d in self.shape:
            n *= int(d)
        return n * torch.empty((), dtype=self.dtype).element_size()


@dataclass
class Node:
    kind: str
    inputs: list
    outputs: list
    slot: int = 0
    attrs: dict = field(default_factory=dict)


class Graph:
    def __init__(self, name: str = "graph"):
        self.name = name
        self.tensors: list[TensorSpec] = []
        self.nodes: list[Node] = []
        self.inputs: list[int] = []
        self.outputs: list[int] = []

    def tensor(self, shape, dtype=torch.bfloat16, name="t", external=False) -> int:
        self.tensors.append(TensorSpec(tuple(int(s) for s in shape), dtype, name, external))
        return len(self.tensors) - 1

    def add(self, kind: str, inputs, outputs, slot: int = 0, **attrs) -> Node:
        n = Node(kind, list(inputs), list(outputs), slot, attrs)
        self.nodes.append(n)
        return n

    def shape(self, tid: int) -> tuple:
        return self.tensors[tid].shape

    def summary(self) -> str:
        kinds: dict[str, int] = {}
        for n in self.nodes:
            kinds[n.kind] = kinds.get(n.kind, 0) + 1
        return f"{self.name}: {len(self.nodes)} nodes {kinds}, {len(self.tensors)} tensors"


def lifetimes(g: Graph) -> dict[int, list[int]]:
    """tensor id -> [first_node, last_node] (internal tensors only)."""
    life: dict[int, list[int]] = {}
    for i, n in enumerate(g.nodes):
        for t in list(n.inputs) + list(n.outputs):
            if t is None or g.tensors[t].external:
                continue
            if t not in life:
                life[t] = [i, i]
            else:
                life[t][0] = min(life[t][0], i)
                life[t][1] = max(life[t][1], i)
    # fork/join windows: anything touched inside lives for the whole window
    stack: dict[int, int] = {}
    windows = []
    for i, n in enumerate(g.nodes):
        if n.kind == "fork":
            stack[n.slot] = i
        elif n.kind == "join" and n.slot in stack:
            windows.append((stack.pop(n.slot), i))
    for (a, b) in windows:
        for t, (s, e) in life.items():
            if s <= b and e >= a:
                life[t] = [min(s, a), max(e, b)]
    return life


def plan_memory(g: Graph, reuse: bool | None = None, groups=()) -> tuple[dict[int, int], int]:
    """Return ({tensor id: arena byte offset}, arena bytes). ``reuse=False`` (or env
    ``HIPZAP_ARENA_NOREUSE=1``) gives every tensor its own slot, so every intermediate stays
    readable after a run (per-node debugging, ``scripts/debug_nodes.py``).
    ``groups``: (first, end) node ranges that run as ONE launch (engine/fusion.py): every tensor
    the range reads or writes is live over the whole range, so a fused kernel's output never
    shares memory with an input its other workgroups still read (a halo) -- the per-node
    lifetimes would let the block output reuse the block input of a downsample block."""
    if reuse is None:
        reuse = os.environ.get("HIPZAP_ARENA_NOREUSE", "0") != "1"
    life = lifetimes(g)
    for first, end in groups:
        for n in g.nodes[first:end]:
            for t in list(n.inputs) + list(n.outputs):
                if t is not None and t in life:
                    life[t] = [min(life[t][0], first), max(life[t][1], end - 1)]
    if not reuse:
        life = {t: [0, len(g.nodes)] for t in life}
    order = sorted(life.keys(), key=lambda t: -g.tensors[t].nbytes)
    placed: list[tuple[int, int, int, int]] = []  # (offset, end, first, last)
    offsets: dict[int, int] = {}
    for t in order:
        size = (g.tensors[t].nbytes + ALIGN - 1) // ALIGN * ALIGN
        s, e = life[t]
        conflicts = sorted((o, oe) for (o, oe, a, b) in placed if a <= e and b >= s)
        off = 0
        for (o, oe) in conflicts:
            if off + size <= o:
                break
            off = max(off, oe)
        offsets[t] = off
        placed.append((off, off + size, s, e))
    total = max([oe for (_, oe, _, _) in placed], default=0)
    return offsets, total
