"""ISA tooling for the CPU tier (test tooling, not product): the gfx950 code objects inside libmapfed.so, their
disassembly, and a static check of the vector-memory wait counts.

``device_disassembly(so_path)`` unbundles the ``.hip_fatbin`` section (clang offload bundles, one per translation
unit) and returns ``llvm-objdump -d`` of every gfx950 code object, split by kernel symbol.

Wait counts:

Every VGPR a global / buffer load writes is "in flight" until an ``s_waitcnt vmcnt(N)`` retires it: the
hardware decrements vmcnt in issue order for loads and stores alike (gfx9 has no separate store counter),
so after ``vmcnt(N)`` all but the N most recent vector-memory operations are complete.  This module walks
every control-flow path of a kernel (the CFG of ``hipcc -S`` output, loops unrolled twice), keeps the
ordered list of outstanding operations, and reports any instruction that reads or overwrites a VGPR whose
load may still be outstanding on some path -- the defect class that makes a result depend on memory
latency.

``check_kernel(asm_text, kernel_name)`` returns a list of hazards (empty when the waits cover every use).
"""

from __future__ import annotations

import re
import struct
import subprocess
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

LLVM_BIN = Path("/opt/rocm/lib/llvm/bin")
_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so_path) -> list[bytes]:
    """The gfx950 code objects (ELF images) of a HIP shared library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as td:
        fat = Path(td) / "fat.bin"
        subprocess.run([str(LLVM_BIN / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(so_path),
                        str(Path(td) / "discard")], check=True, capture_output=True)
        data = fat.read_bytes()
    out, i = [], 0
    while True:
        i = data.find(_BUNDLE_MAGIC, i)
        if i < 0:
            return out
        (n,) = struct.unpack_from("<Q", data, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple and size:
                out.append(data[i + off:i + off + size])
        i += len(_BUNDLE_MAGIC)


def device_disassembly(so_path) -> dict[str, list[str]]:
    """kernel symbol -> its disassembled instruction lines, over every gfx950 code object of the library."""
    kernels: dict[str, list[str]] = {}
    with tempfile.TemporaryDirectory() as td:
        for n, co in enumerate(code_objects(so_path)):
            f = Path(td) / f"co{n}.elf"
            f.write_bytes(co)
            txt = subprocess.run([str(LLVM_BIN / "llvm-objdump"), "-d", "--no-show-raw-insn", str(f)], check=True,
                                 capture_output=True, text=True).stdout
            cur = None
            for ln in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:$", ln)
                if m:
                    cur = m.group(1)
                    kernels[cur] = []
                elif cur is not None and ln.strip():
                    kernels[cur].append(ln.strip())
    return kernels

_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_WAIT = re.compile(r"vmcnt\((\d+)\)")
_LABEL = re.compile(r"^(\.LBB\w+|\.L\w+):")
# vector-memory instructions that write VGPRs when they return (first operand = destination)
_VMEM_LOAD = re.compile(r"^(global_load|buffer_load|flat_load|global_atomic\w*_rtn|buffer_atomic\w*_rtn|scratch_load)")
_VMEM_STORE = re.compile(r"^(global_store|buffer_store|flat_store|scratch_store|global_atomic(?!.*_rtn)|buffer_atomic)")
# instructions whose every operand is a source (no VGPR destination)
_NO_VDST = re.compile(r"^(s_|ds_write|ds_store|global_store|buffer_store|flat_store|scratch_store|v_cmp|v_cmpx|exp\b)")


def _regs(text: str) -> set[int]:
    out: set[int] = set()
    for m in _VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


@dataclass
class Inst:
    line: int
    text: str
    op: str
    dst: set[int] = field(default_factory=set)
    src: set[int] = field(default_factory=set)


@dataclass
class Block:
    label: str
    insts: list[Inst] = field(default_factory=list)
    succ: list[str] = field(default_factory=list)


def kernel_body(asm: str, name: str) -> list[tuple[int, str]]:
    """Lines of one kernel's function body (from its label to s_endpgm's section end)."""
    lines = asm.splitlines()
    start = None
    for i, ln in enumerate(lines):
        if ln.startswith(name + ":"):
            start = i + 1
            break
    if start is None:
        raise KeyError(name)
    body = []
    for i in range(start, len(lines)):
        ln = lines[i]
        if ln.lstrip().startswith(".section") or ln.startswith(".Lfunc_end"):
            break
        body.append((i + 1, ln))
    return body


def parse_blocks(body: list[tuple[int, str]]) -> tuple[list[Block], dict[str, int]]:
    blocks: list[Block] = [Block("<entry>")]
    for lineno, raw in body:
        s = raw.split(";")[0].strip()
        if not s:
            continue
        m = _LABEL.match(s)
        if m:
            blocks.append(Block(m.group(1)))
            continue
        if s.startswith("."):
            continue
        op = s.split()[0]
        args = s[len(op):]
        inst = Inst(lineno, s, op)
        if _VMEM_STORE.match(op) or _NO_VDST.match(op):
            inst.src = _regs(args)
        else:
            first, _, rest = args.partition(",")
            inst.dst = _regs(first)
            inst.src = _regs(rest)
            if op.startswith("v_mfma") or op.startswith("v_dot") or "_mac_" in op or op.startswith("v_fmac"):
                inst.src |= inst.dst  # accumulating forms read their destination
        blocks[-1].insts.append(inst)
        if op == "s_endpgm" or op == "s_branch" or op.startswith("s_cbranch") or op == "s_setpc_b64":
            blocks.append(Block(f"<after {lineno}>"))
    blocks = [b for b in blocks if b.insts or b.label.startswith(".")]
    index = {b.label: i for i, b in enumerate(blocks)}
    for i, b in enumerate(blocks):
        last = b.insts[-1] if b.insts else None
        fall = blocks[i + 1].label if i + 1 < len(blocks) else None
        if last is None:
            b.succ = [fall] if fall else []
        elif last.op == "s_endpgm":
            b.succ = []
        elif last.op == "s_branch":
            b.succ = [last.text.split()[1]]
        elif last.op.startswith("s_cbranch"):
            b.succ = [last.text.split()[1]] + ([fall] if fall else [])
        else:
            b.succ = [fall] if fall else []
    return blocks, index


def check_kernel(asm: str, name: str, max_visits: int = 2) -> list[str]:
    """Walk every path; report reads/overwrites of VGPRs with a possibly outstanding load."""
    blocks, index = parse_blocks(kernel_body(asm, name))
    hazards: dict[int, str] = {}
    seen: set[tuple[int, tuple]] = set()
    # state: tuple of outstanding ops, oldest first; each op = frozenset of destination VGPRs (empty = store)
    work: list[tuple[int, tuple, tuple]] = [(0, (), ())]
    while work:
        bi, pend, visits = work.pop()
        key = (bi, pend)
        if key in seen:
            continue
        seen.add(key)
        pend_l = list(pend)
        for inst in blocks[bi].insts:
            if inst.op == "s_waitcnt":
                m = _WAIT.search(inst.text)
                if m:
                    n = int(m.group(1))
                    while len(pend_l) > n:
                        pend_l.pop(0)
                continue
            if pend_l:
                inflight = set().union(*pend_l)
                bad = (inst.src | inst.dst) & inflight
                if bad and inst.line not in hazards:
                    hazards[inst.line] = f"line {inst.line}: {inst.text}  (v{sorted(bad)} may still be loading)"
            if _VMEM_LOAD.match(inst.op):
                pend_l.append(frozenset(inst.dst))
            elif _VMEM_STORE.match(inst.op):
                pend_l.append(frozenset())
        nv = visits + (bi,)
        for s in blocks[bi].succ:
            if s not in index:
                continue
            si = index[s]
            if nv.count(si) >= max_visits:
                continue
            work.append((si, tuple(pend_l), nv if si <= bi else visits))
    return [hazards[k] for k in sorted(hazards)]


def kernel_names(asm: str, pattern: str) -> list[str]:
    return [m.group(1) for m in re.finditer(r"^(_Z\S*" + pattern + r"\S*):", asm, re.M)]
