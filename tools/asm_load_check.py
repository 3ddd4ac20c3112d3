"""Mechanical check of the inline-asm register loads.

Some kernels load global memory into VGPRs from inline asm (the GEMM's register weight slices `ldw32` / `ldw64`,
the residual epilogue's row loads, the UltraNet tail's weight prefetch `fetch_w`) and wait for them with counted
`s_waitcnt vmcnt(N)`, because a compiler-visible load would make the compiler drain the asm-issued LDS-DMA stream.
The compiler treats such a destination as written when the asm returns, although the data only lands at the
counted wait. Each site therefore ends in a "pin": an asm statement that takes the registers as "+v" operands
after the wait, so no use of them can be scheduled above it. What the pin cannot stop is the compiler touching
the registers between the load and the pin (a copy, a spill, a reuse). This tool checks exactly that on the
compiler's device assembly, for every load on every control-flow path:

  * the load asm carries the marker comment `; qvit_asm_load`, the pin asm `; qvit_pin <its registers>`;
  * from each marked load, every path must reach an `s_waitcnt vmcnt(N)` that covers the load (N no larger than
    the vector-memory operations issued after the load on that path) before any instruction mentions one of the
    load's destination registers: no read, copy, spill, overwrite or pin of them while the data is in flight.

The walk follows every control-flow path except those whose uniform branch conditions contradict each other (one
condition mask tested twice, or a mask the compiler set to a constant; `_branch_facts`), so it can only over-report.

    python tools/asm_load_check.py FILE.s [...]      (device assembly: hipcc --cuda-device-only -S)
"""
from __future__ import annotations

import re
import sys
from dataclasses import dataclass, field

_VREG = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)\b)")
_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
_FUNC = re.compile(r"^(_Z\S+):")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")
_VMEM = ("global_", "buffer_", "scratch_", "flat_")


def vregs(text: str) -> set:
    out = set()
    for m in _VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


@dataclass
class Ins:
    line: int           # 1-based line in the .s file
    text: str           # instruction without comment
    op: str
    load_mark: bool = False   # inside a `; qvit_asm_load` asm block
    pin: set = field(default_factory=set)   # registers a `; qvit_pin` names (empty: not a pin)
    vr: frozenset = frozenset()   # the VGPRs the instruction mentions (set by parse)
    sd: object = None             # the scalar register it writes, if any (set by parse)


@dataclass
class Func:
    name: str
    ins: list
    labels: dict   # label -> index of the next instruction


def parse(path: str) -> list:
    funcs, cur = [], None
    in_asm, asm_load, asm_pin = False, False, set()
    with open(path) as f:
        lines = f.read().split("\n")
    for i, raw in enumerate(lines, 1):
        s = raw.strip()
        m = _FUNC.match(raw)
        if m:
            cur = Func(m.group(1), [], {})
            funcs.append(cur)
            continue
        if cur is None:
            continue
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        if s == ";;#ASMSTART":
            in_asm, asm_load, asm_pin = True, False, set()
            continue
        if s == ";;#ASMEND":
            if asm_pin:   # a pin block: one pseudo instruction at its end (after any wait it holds)
                cur.ins.append(Ins(i, "", "qvit_pin", pin=asm_pin))
            in_asm = False
            continue
        m = _LABEL.match(s)
        if m:
            cur.labels[m.group(1)] = len(cur.ins)
            continue
        if not s or s.startswith(";") and not in_asm or s.startswith("."):
            continue
        if s.startswith(";"):
            if "qvit_asm_load" in s:
                asm_load = True
            elif "qvit_pin" in s:
                asm_pin = vregs(s)
            continue
        text = s.split(";")[0].strip()
        if not text:
            continue
        op = text.split()[0]
        cur.ins.append(Ins(i, text, op, load_mark=in_asm and asm_load and op.startswith(_VMEM)))
    for fn in funcs:
        for x in fn.ins:
            x.vr = frozenset(x.pin) if x.pin else frozenset(vregs(x.text))
            x.sd = _sdst(x)
    return funcs


def _succ(fn: Func, k: int):
    ins = fn.ins[k]
    if ins.op == "s_endpgm" or ins.op.startswith("s_setpc"):
        return []
    if ins.op == "s_branch":
        return [fn.labels[ins.text.split()[1]]]
    if ins.op.startswith("s_cbranch"):
        return [k + 1, fn.labels[ins.text.split()[1]]]
    return [k + 1]


_SDST = re.compile(r"^(s\[\d+:\d+\]|s\d+|vcc|exec)(?!\w)")
_NO_SDST = ("s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_setprio", "s_cmp", "s_bitcmp",
            "s_endpgm", "s_sleep", "s_sendmsg", "s_dcache", "s_icache", "s_trap", "s_setpc", "s_swappc")


def _sdst(ins: Ins):
    """The scalar register an instruction writes (its first operand), if any."""
    if ins.op.startswith(_NO_SDST) or not (ins.op.startswith("s_") or ins.op.startswith("v_cmp")
                                           or ins.op.startswith("v_read")):
        return None
    ops = ins.text[len(ins.op):].strip()
    m = _SDST.match(ops)
    return m.group(1) if m else None


def _tested_masks(fn: Func) -> set:
    """Condition masks the function tests more than once, or sets to a constant and tests: the only ones whose
    facts can prune a path (keeping no others bounds the walk's states)."""
    tests, consts = {}, set()
    for x in fn.ins:
        if x.op in ("s_and_b64", "s_andn2_b64") and x.text.split(",")[0].split()[-1] == "vcc":
            parts = [p.strip() for p in x.text[len(x.op):].split(",")]
            if len(parts) == 3 and parts[1] == "exec":
                tests[parts[2]] = tests.get(parts[2], 0) + 1
        elif x.op == "s_mov_b64":
            parts = [p.strip() for p in x.text[len(x.op):].split(",")]
            if len(parts) == 2 and parts[1] in ("-1", "0"):
                consts.add(parts[0])
    return {r for r, n in tests.items() if n > 1 or r in consts}


def _branch_facts(fn: Func, k: int, facts: frozenset, keep: set):
    """Successors of instruction k with the uniform branch facts each one implies, infeasible ones dropped.
    A fact is (register, value): a wave-uniform condition mask the compiler tested (`s_and_b64 vcc, exec, R` or
    `s_andn2_b64 vcc, exec, R` then `s_cbranch_vcc[n]z`), or a mask it set to a constant (`s_mov_b64 R, -1 / 0`).
    Tracking them prunes the paths through correlated branches (one condition tested twice) that never run."""
    ins = fn.ins[k]
    d = dict(facts)
    dst = ins.sd
    if ins.op == "s_mov_b64" and dst:
        src = ins.text.split(",")[1].strip()
        d.pop(dst, None)
        if dst in keep and src in ("-1", "0"):
            d[dst] = src == "-1"
        elif dst in keep and src in d:
            d[dst] = d[src]
    elif ins.op in ("s_and_b64", "s_andn2_b64") and dst == "vcc" and ins.text.split(",")[1].strip() == "exec":
        src = ins.text.split(",")[2].strip()
        d.pop("vcc", None)
        if src in keep:
            d["vcc"] = ("cond", src, ins.op == "s_and_b64")
    elif dst:
        d.pop(dst, None)
        for r in [r for r, v in d.items() if isinstance(v, tuple) and v[1] == dst]:
            d.pop(r)
    out = []
    nxt = _succ(fn, k)
    if ins.op in ("s_cbranch_vccnz", "s_cbranch_vccz") and isinstance(d.get("vcc"), tuple):
        _, src, pol = d["vcc"]
        for j, n in enumerate(nxt):
            taken = j == 1
            val = pol if (taken == (ins.op == "s_cbranch_vccnz")) else not pol   # the value of src on this edge
            if src in d and d[src] != val:
                continue   # contradicts what this path already established: never runs
            e = dict(d)
            e[src] = val
            out.append((n, frozenset(e.items())))
        return out
    return [(n, frozenset(d.items())) for n in nxt]


def _walk(fn: Func, k0: int, cap: int, keep):
    """Violations of the load at instruction k0 on the paths from it; keep = None: every path (fast), else the
    paths whose tested condition masks in `keep` agree with each other."""
    ld, errs = fn.ins[k0], []
    pend = frozenset(vregs(ld.text.split(",")[0]))
    stack = [(k0 + 1, 0, frozenset())]
    seen = set()
    while stack:
        k, cnt, facts = stack.pop()
        while True:
            if (k, cnt, facts) in seen:
                break
            seen.add((k, cnt, facts))
            if k >= len(fn.ins):
                errs.append(f"{fn.name}: load at line {ld.line} falls off the function unwaited")
                break
            ins = fn.ins[k]
            if pend & ins.vr:
                what = "its pin" if ins.pin else f"`{ins.text}`"
                errs.append(f"{fn.name}: load at line {ld.line}: line {ins.line} ({what}) touches its "
                            f"destination before a covering s_waitcnt vmcnt ({cnt} younger operations)")
                break
            if ins.op.startswith(_VMEM):
                cnt = min(cnt + 1, cap)
            elif ins.op == "s_waitcnt":
                m = _VMCNT.search(ins.text)
                if m and int(m.group(1)) <= cnt:
                    break   # landed on this path: any later use, copy or reuse of the registers is safe
            elif ins.op == "s_endpgm":
                errs.append(f"{fn.name}: load at line {ld.line} reaches s_endpgm unwaited (line {ins.line})")
                break
            if keep is None:
                nxt = [(n, facts) for n in _succ(fn, k)]
            else:
                nxt = _branch_facts(fn, k, facts, keep)
            if not nxt:
                break
            stack.extend((n, cnt, f) for n, f in nxt[1:])
            k, facts = nxt[0]
    return sorted(set(errs))


def check_func(fn: Func):
    """-> (number of marked loads, list of violation strings)"""
    errs, nloads, keep = [], 0, None
    # counts beyond the largest vmcnt operand in the function all behave alike
    cap = 1 + max([int(m.group(1)) for x in fn.ins if x.op == "s_waitcnt" for m in [_VMCNT.search(x.text)] if m]
                  + [0])
    for k0, ld in enumerate(fn.ins):
        if not ld.load_mark:
            continue
        nloads += 1
        e = _walk(fn, k0, cap, None)
        if e:   # again on the feasible paths only (correlated branches pruned)
            if keep is None:
                keep = _tested_masks(fn)
            e = _walk(fn, k0, cap, keep)
        errs += e
    return nloads, errs


def check_file(path: str):
    """-> ({function: marked loads}, [violations])"""
    counts, errs = {}, []
    for fn in parse(path):
        n, e = check_func(fn)
        if n:
            counts[fn.name] = n
        errs += e
    return counts, errs


def main(argv):
    bad = 0
    for path in argv:
        counts, errs = check_file(path)
        print(f"{path}: {sum(counts.values())} asm loads in {len(counts)} kernels")
        for e in errs:
            print("  VIOLATION", e)
        bad += len(errs)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
