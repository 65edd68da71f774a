"""Static wait-counter hazard check over compiled gfx950 ISA (a development and
test helper; see tests/test_asm_pipeline.py).

  hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S f.hip -o f.s
  python tools/isa_hazard_check.py f.s [kernel-substring ...]

What it models, per wave, over the kernel's control-flow graph (basic blocks
from labels and branches, every branch both ways, loops to a fixed point):

* the vector-memory queue (vmcnt): every global_/buffer_/scratch_ load,
  store and atomic, in issue order (gfx950 has no separate store counter).
  `s_waitcnt vmcnt(N)` retires an op once N ops were issued after it on EVERY
  path to the wait (the state keeps, per pending op, the minimum over paths of
  the ops issued after it);
* the LDS / scalar-memory queue (lgkmcnt): ds_* ops retire in order among
  themselves, s_load_* (out of order) only at lgkmcnt(0);
* LDS-DMA loads (`... lds`) as a pending write to LDS;
* the LDS hand-off at `s_barrier`: other waves read what this wave wrote to
  LDS before the barrier, and write what it read, so a ds_write / LDS-DMA
  still in flight at a barrier is a hazard, and so is a ds_read in flight.

Hazards reported: any instruction reading a register (v, a or s) a pending
load will still write (RAW); any instruction other than a load of the same
in-order queue writing such a register (WAW: the load lands later and
clobbers it); the barrier hand-offs above.  Inline asm (`;;#ASMSTART`) is
treated like compiled code: the point is to check hand-counted waits
(spmm_hub_kernel, dense_kernel) together with everything hipcc emitted.

Exec-masked row loads (round 5; check_kernel(exec_rule=True)): a 16-byte VMEM load (a row gather or a
record / item descriptor) issued while exec is not known to be full (inside
an s_and_saveexec region or a divergent loop) writes only the active lanes;
the other lanes keep the register's older value.  If such a register is then
read as data (a floating-point / select / MFMA / packed op, not address
arithmetic) after exec was widened again (s_or_b64 / s_mov_b64 / s_xor_b64
exec: the join of a divergent region) and before anything rewrote it, a
partial write crosses a join -- the pattern of the round-4 fused kernels'
prefetch (`if (u < pn) vload(pv[u], ...)`, folded at the next tile).  The
hardware does what the ISA says here; the rule marks a form whose
correctness rests on the register allocator keeping the masked lanes, which
the 128-wide fused kernels now avoid (every gather and descriptor load is
issued with full exec; absent edges read kgx_zero_row).  Reported as "data
read of a register an exec-masked 16-byte load wrote, after an exec join"
(tests/test_asm_pipeline.py holds those kernels to zero).

Not modelled: which lanes a mask holds (any partial exec counts), partial
writes by VALU instructions (loop-carried sums under a divergent loop are the
compiler's ordinary phis), instruction-level hazards the hardware resolves by
s_nop (VALU -> DPP / MFMA forwarding), and which LDS bytes a barrier actually
hands off (any LDS op in flight at a barrier counts).
"""

from __future__ import annotations

import re
import sys
from collections import defaultdict

CAP = 64  # waitcnt fields are < 64: counts past this behave the same


def parse_regs(tok: str) -> set:
    tok = tok.strip()
    m = re.match(r"^([vsa])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"^([vsa])(\d+)\b", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    if tok.startswith(("vcc", "exec")):
        return set()
    return set()


def operands(line: str) -> tuple[str, list]:
    parts = line.split(None, 1)
    op = parts[0]
    if len(parts) == 1:
        return op, []
    toks = [t.strip() for t in re.split(r",(?![^\[]*\])", parts[1])]
    return op, toks


def classify(op: str, line: str) -> str:
    if op.startswith(("global_load", "buffer_load", "scratch_load", "flat_load")):
        return "vmem_lds" if re.search(r"\blds\b", line) else "vmem_load"
    if op.startswith(("global_store", "buffer_store", "scratch_store", "flat_store")):
        return "vmem_store"
    if op.startswith(("global_atomic", "buffer_atomic", "flat_atomic")):
        return "vmem_atomic_ret" if re.search(r"\b(glc|sc0)\b", line) else "vmem_store"
    if op.startswith("ds_"):
        if op.startswith(("ds_write", "ds_store")) or (op.startswith(("ds_add", "ds_max", "ds_min", "ds_and", "ds_or"))
                                                       and "_rtn" not in op):
            return "ds_write"
        return "ds_read"
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_dcache", "s_scratch_load")):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op == "s_barrier":
        return "barrier"
    return "alu"


class State:
    """vm: {reg: younger-op count}; vm_n: younger counts of pending LDS-DMA ops;
    ds: {reg: younger LDS-op count}; ds_w / ds_r: pending LDS writes / reads
    (younger LDS-op counts); sm: regs of pending scalar loads."""

    __slots__ = ("vm", "vm_n", "ds", "ds_w", "ds_r", "sm", "pm", "ex", "line")

    def __init__(self):
        self.vm, self.vm_n = {}, frozenset()
        self.ds, self.ds_w, self.ds_r = {}, frozenset(), frozenset()
        self.sm = set()
        self.pm = {}  # reg -> (crossed a join out of its region, load line, region depth): exec-masked load dst
        self.ex = ()  # exec narrowings in force (saved-mask pairs / "n"); () = every lane of the wave on
        self.line = -1

    def copy(self):
        s = State()
        s.vm, s.vm_n = dict(self.vm), self.vm_n
        s.ds, s.ds_w, s.ds_r = dict(self.ds), self.ds_w, self.ds_r
        s.sm = set(self.sm)
        s.pm = dict(self.pm)
        s.ex = self.ex
        return s

    def key(self):
        return (tuple(sorted(self.vm.items())), tuple(sorted(self.vm_n)), tuple(sorted(self.ds.items())),
                tuple(sorted(self.ds_w)), tuple(sorted(self.ds_r)), tuple(sorted(self.sm)),
                tuple(sorted(self.pm.items())), self.ex)

    def join(self, o: "State") -> "State":
        """Pending on either path; younger counts: the minimum (the worst case)."""
        s = State()
        for a, b, out in ((self.vm, o.vm, s.vm), (self.ds, o.ds, s.ds)):
            for r in set(a) | set(b):
                out[r] = min(a.get(r, (CAP, -1)), b.get(r, (CAP, -1)))
        # pending LDS writes / reads / LDS-DMA: the sets of their younger counts
        # (only whether one is pending matters, and a wait retires by count)
        for name in ("vm_n", "ds_w", "ds_r"):
            setattr(s, name, getattr(self, name) | getattr(o, name))
        s.sm = self.sm | o.sm
        for r in set(self.pm) | set(o.pm):
            s.pm[r] = max(self.pm.get(r, (False, -1, 0)), o.pm.get(r, (False, -1, 0)))
        s.ex = max(self.ex, o.ex, key=lambda e: (len(e), str(e)))  # the more narrowed (conservative)
        return s


# data uses (not address arithmetic): float / select / conversion / packed / matrix ops
_DATA_READ = re.compile(r"^v_(\w*_f32|\w*_f16|\w*bf16\w*|cndmask\w*|pk_\w+|mfma\w*|max\w*|min\w*|med3\w*|perm\w*)")
_EXEC_WIDEN = ("s_or_b64", "s_mov_b64", "s_xor_b64", "s_or_saveexec_b64", "s_andn2_saveexec_b64", "s_not_b64")


def _exec_step(st: State, op: str, toks: list, line: str, report) -> None:
    """The exec-masked load rule (module docstring): reads of crossed registers,
    then this instruction's effect on the partial-write set."""
    kind = classify(op, line)
    if not toks or kind == "wait":
        return
    load = kind in ("vmem_load", "vmem_atomic_ret")
    writes_dst = kind in ("vmem_load", "vmem_atomic_ret", "ds_read") or (
        kind in ("alu", "smem") and not op.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_nop", "s_set",
                                                      "s_sleep", "s_endpgm", "s_sendmsg", "s_waitcnt", "s_barrier")))
    dst = parse_regs(toks[0]) if writes_dst else set()
    srcs = set()
    for t in (toks[1:] if writes_dst else toks):
        srcs |= parse_regs(t)
    if op.startswith("v_pk_") and writes_dst:
        srcs = _pk_sources(toks, line)
    crossed = sorted(r for r in srcs if st.pm.get(r, (False,))[0])
    if crossed and _DATA_READ.match(op):
        report("data read of a register an exec-masked 16-byte load wrote, after an exec join"
               f" [loads at lines {sorted({st.pm[r][1] for r in crossed})}]", line)
    for r in dst:
        st.pm.pop(r, None)
    if load and st.ex and len(dst) >= 4:
        for r in dst:
            st.pm[r] = (False, st.line, len(st.ex))
    # the structured exec stack hipcc emits: s_and_saveexec s[x] opens a region,
    # s_and(n2)_b64 exec, exec, .. narrows (divergent loops, masked stores),
    # s_or_b64 exec, exec, s[x] / s_mov_b64 exec, s[x] closes back to x
    if op in ("s_and_saveexec_b64", "s_andn2_saveexec_b64", "s_or_saveexec_b64"):
        x = _pair(toks[0])
        ex = list(st.ex)
        if op != "s_and_saveexec_b64" and ex:
            # the else branch of the region just opened (s_and_saveexec s[y]; s_xor
            # s[x], exec, s[y]; s_andn2_saveexec s[x], s[x]): s[x] now closes it
            ex = ex[:-1]
        st.ex = (tuple(ex) + (x,))[-6:]  # bounded (a fixed point over loops)
    elif toks[0] == "exec":
        if op in ("s_and_b64", "s_andn2_b64"):
            if not st.ex or st.ex[-1] != "n":  # a divergent loop narrows once per iteration: one entry
                st.ex = (st.ex + ("n",))[-6:]
        else:
            x = _pair(toks[2]) if op == "s_or_b64" and len(toks) == 3 else (_pair(toks[1]) if len(toks) == 2 else None)
            ex = list(st.ex)
            if x in ex:
                ex = ex[: ex.index(x)]
            else:  # a loop's exit mask (not a saved region): undo the loop's narrowing
                while ex and ex[-1] == "n":
                    ex.pop()
            st.ex = tuple(ex)
        if op in _EXEC_WIDEN and st.pm:  # a join that leaves the load's region: the value crosses it
            d = len(st.ex)
            st.pm = {r: (c or d < dep, ln, dep) for r, (c, ln, dep) in st.pm.items()}


def step(st: State, line: str, report, exec_rule: bool = False) -> State:
    op, toks = operands(line)
    if exec_rule:
        _exec_step(st, op, toks, line, report)
    kind = classify(op, line)
    pend = set(st.vm) | set(st.ds) | st.sm
    if kind == "wait":
        m = re.search(r"vmcnt\((\d+)\)", line)
        if m:
            n = int(m.group(1))
            st.vm = {r: y for r, y in st.vm.items() if y[0] < n}
            st.vm_n = frozenset(y for y in st.vm_n if y < n)
        m = re.search(r"lgkmcnt\((\d+)\)", line)
        if m:
            n = int(m.group(1))
            st.ds = {r: y for r, y in st.ds.items() if y[0] < n}
            st.ds_w = frozenset(y for y in st.ds_w if y < n)
            st.ds_r = frozenset(y for y in st.ds_r if y < n)
            if n == 0:
                st.sm = set()
        if re.fullmatch(r"s_waitcnt\s+0", line.strip()):
            st.vm, st.vm_n, st.ds, st.ds_w, st.ds_r, st.sm = {}, frozenset(), {}, frozenset(), frozenset(), set()
        return st
    if kind == "barrier":
        if st.ds_w:
            report("LDS write in flight at s_barrier (other waves read it after the barrier)", line)
        if st.ds_r:
            report("LDS read in flight at s_barrier (other waves may overwrite its bytes after it)", line)
        if st.vm_n:
            report("LDS-DMA load in flight at s_barrier", line)
        return st
    if not toks:
        return st
    if kind in ("vmem_load", "vmem_lds", "vmem_store", "vmem_atomic_ret"):
        dst = parse_regs(toks[0]) if kind in ("vmem_load", "vmem_atomic_ret") else set()
        srcs = set()
        for t in (toks[1:] if kind in ("vmem_load", "vmem_atomic_ret") else toks):
            srcs |= parse_regs(t)
        if kind == "vmem_lds":
            srcs = set()
            for t in toks:
                srcs |= parse_regs(t)
        if srcs & pend:
            report("address/data reads a register a pending load will write", line)
        if dst & (set(st.ds) | st.sm):
            report("VMEM load into a register a pending LDS/scalar load will write (no order between queues)", line)
        st.vm = {r: (min(y + 1, CAP), src) for r, (y, src) in st.vm.items()}
        st.vm_n = frozenset(min(y + 1, CAP) for y in st.vm_n) | (frozenset([0]) if kind == "vmem_lds" else frozenset())
        for r in dst:
            st.vm[r] = (0, st.line)
        return st
    if kind in ("ds_read", "ds_write"):
        dst = parse_regs(toks[0]) if kind == "ds_read" else set()
        srcs = set()
        for t in (toks[1:] if kind == "ds_read" else toks):
            srcs |= parse_regs(t)
        if srcs & pend:
            report("LDS op reads a register a pending load will write", line)
        if dst & (set(st.vm) | st.sm):
            report("LDS read into a register a pending VMEM/scalar load will write (no order between queues)", line)
        st.ds = {r: (min(y + 1, CAP), src) for r, (y, src) in st.ds.items()}
        st.ds_w = frozenset(min(y + 1, CAP) for y in st.ds_w)
        st.ds_r = frozenset(min(y + 1, CAP) for y in st.ds_r)
        for r in dst:
            st.ds[r] = (0, st.line)
        if kind == "ds_write":
            st.ds_w = st.ds_w | {0}
        else:
            st.ds_r = st.ds_r | {0}
        return st
    if kind == "smem":
        dst = parse_regs(toks[0]) if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime")) else set()
        srcs = set()
        for t in toks[1:]:
            srcs |= parse_regs(t)
        if srcs & pend:
            report("scalar load address reads a register a pending load will write", line)
        st.sm |= dst
        return st
    # ALU (VALU, MFMA, SALU, readlane, ...): operand 0 is the destination except
    # for compares / branches / no-destination forms
    no_dst = op.startswith(("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_setprio", "s_nop", "s_sleep",
                            "s_endpgm", "s_setpc", "s_sendmsg", "s_set", "s_ttrace", "s_trap", "s_icache"))
    dst = set() if no_dst else parse_regs(toks[0])
    srcs = set()
    for t in (toks if no_dst else toks[1:]):
        srcs |= parse_regs(t)
    if op.startswith("v_pk_") and not no_dst:
        srcs = _pk_sources(toks, line)
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        pass  # srcC (the last operand) is read like the others
    if srcs & pend:
        report("read of a register a pending load will write" + _src(st, srcs & pend), line)
    if dst & pend:
        report("write to a register a pending load will write (the load lands later)" + _src(st, dst & pend), line)
    return st


def _pk_sources(toks: list, line: str) -> set:
    """Registers a packed (v_pk_*) instruction reads: of a 64-bit source pair,
    the low lane reads the low register unless op_sel picks the high one, the
    high lane the high register unless op_sel_hi picks the low one."""
    def sel(name, n, default):
        m = re.search(name + r":\[([01,]+)\]", line)
        v = [int(x) for x in m.group(1).split(",")] if m else [default] * n
        return v + [default] * (n - len(v))
    srcs_t = [t for t in toks[1:] if re.match(r"^[vsa]\[|^[vsa]\d", t)]
    lo_sel, hi_sel = sel(r"\bop_sel", len(srcs_t), 0), sel("op_sel_hi", len(srcs_t), 1)
    out = set()
    for i, t in enumerate(srcs_t):
        regs = sorted(parse_regs(t))
        if len(regs) == 2:
            out.add(regs[lo_sel[i]])
            out.add(regs[hi_sel[i]])
        else:
            out |= set(regs)
    return out


def _src(st, regs) -> str:
    lines = sorted({(st.vm.get(r) or st.ds.get(r) or (0, -1))[1] for r in regs})
    return f" [loads at lines {lines}]"


def build_cfg(lines: list):
    """Basic blocks: (start, end) line ranges and successor block ids."""
    starts = {0}
    labels = {}
    for k, l in enumerate(lines):
        if re.match(r"^\.?\w[\w.]*:$", l):
            labels[l[:-1]] = k
            starts.add(k)
        op = l.split()[0] if l else ""
        if op.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            starts.add(k + 1)
    starts = sorted(s for s in starts if s < len(lines))
    blocks = [(a, b) for a, b in zip(starts, starts[1:] + [len(lines)])]
    index = {a: i for i, (a, _) in enumerate(blocks)}
    succ = defaultdict(list)
    for i, (a, b) in enumerate(blocks):
        last = next((lines[k] for k in range(b - 1, a - 1, -1) if lines[k] and not lines[k].endswith(":")), "")
        op = last.split()[0] if last else ""
        if op.startswith(("s_branch", "s_cbranch")):
            tgt = last.split()[1] if len(last.split()) > 1 else None
            if tgt in labels:
                succ[i].append(index[labels[tgt]])
            if op.startswith("s_cbranch") and i + 1 < len(blocks):
                succ[i].append(i + 1)
        elif op.startswith(("s_endpgm", "s_setpc")):
            pass
        elif i + 1 < len(blocks):
            succ[i].append(i + 1)
    return blocks, succ


def _pair(tok: str):
    m = re.match(r"^s\[(\d+):(\d+)\]$", tok.strip())
    return int(m.group(1)) if m and int(m.group(2)) == int(m.group(1)) + 1 else None


_CMP = {"eq": lambda a, b: a == b, "lg": lambda a, b: a != b, "gt": lambda a, b: a > b,
        "ge": lambda a, b: a >= b, "lt": lambda a, b: a < b, "le": lambda a, b: a <= b}


def _sconst(f: dict, tok: str):
    """The set of values an SGPR / literal may hold (None: unknown)."""
    tok = tok.strip()
    m = re.match(r"^s(\d+)$", tok)
    if m:
        return f.get(("c", int(m.group(1))))
    try:
        return frozenset([int(tok, 0)])
    except ValueError:
        return None


def flags_step(flags: dict, line: str) -> dict:
    """Scalar flag constants, for the branch correlation hipcc builds loop exits
    from (s_mov_b64 s[x], -1/0 ... s_andn2_b64 vcc, exec, s[x] ... s_cbranch_vcc*):
    64-bit SGPR pairs holding 0 or -1, vcc known zero / non-zero (exec is
    assumed non-zero where a vcc branch is taken on it), and whether exec is
    known full (kernel entry; restored by s_or_b64 / s_mov_b64 exec from a
    mask saved while it was full), so execz / execnz branches there resolve."""
    op, toks = operands(line)
    if op.startswith(("s_cmp_", "s_cmpk_")) and len(toks) == 2:
        f = dict(flags)
        f.pop("scc", None)
        a, b = _sconst(f, toks[0]), _sconst(f, toks[1])
        cmp = op.split("_")[2]
        if a is not None and b is not None and cmp in _CMP:
            m = 0xFFFFFFFF if op.endswith(("u32", "u64")) else -1
            res = {int(_CMP[cmp](x & m if m > 0 else x, y & m if m > 0 else y)) for x in a for y in b}
            if len(res) == 1:
                f["scc"] = res.pop()
        return f
    if not toks or op.startswith(("s_bitcmp", "s_cbranch", "s_branch", "s_nop", "s_waitcnt", "s_barrier")):
        return flags
    f = dict(flags)
    d = toks[0]
    if op.startswith("s_") and not op.startswith(("s_mov", "s_cselect", "s_load", "s_buffer", "s_setprio", "s_sleep")):
        f.pop("scc", None)  # SALU arithmetic / logic writes SCC
    if op == "s_cselect_b64" and _pair(d) is not None and len(toks) == 3 and "scc" in f:
        pick = toks[1] if f["scc"] else toks[2]
        x = _pair(d)
        for r in [k for k in f if k == x or k == ("c", x) or k == ("c", x + 1)]:
            f.pop(r)
        if pick in ("-1", "0"):
            f[x] = int(pick)
        return f
    if op in ("s_mov_b32", "s_movk_i32") and len(toks) == 2 and re.match(r"^s\d+$", d):
        f.pop(("c", int(d[1:])), None)
        v = _sconst(f, toks[1])
        if v is not None:
            f[("c", int(d[1:]))] = v
        return f
    if op == "s_cselect_b32" and len(toks) == 3 and re.match(r"^s\d+$", d):
        a, b = _sconst(f, toks[1]), _sconst(f, toks[2])
        f.pop(("c", int(d[1:])), None)
        v = (a if f["scc"] else b) if "scc" in f else (a | b if a is not None and b is not None else None)
        if v is not None:
            f[("c", int(d[1:]))] = v
        return f
    if op == "s_and_saveexec_b64" or op == "s_andn2_saveexec_b64":  # entering a divergent region
        x = _pair(d)
        for r in [k for k in f if isinstance(k, int) or (isinstance(k, tuple) and k[0] == "sv")]:
            if r == x or (isinstance(r, tuple) and r[1] == x):
                f.pop(r)
        if f.get("exec") == "full" and x is not None:
            f[("sv", x)] = "full"
        f.pop("exec", None)
        return f
    if d == "exec":
        x = _pair(toks[2]) if op == "s_or_b64" and len(toks) == 3 and toks[1] == "exec" else (
            _pair(toks[1]) if op == "s_mov_b64" and len(toks) == 2 else None)
        f.pop("exec", None)
        if x is not None and f.get(("sv", x)) == "full":
            f["exec"] = "full"
        return f
    if d.startswith("vcc") or d == "vcc":
        f.pop("vcc", None)
        if op in ("s_and_b64", "s_andn2_b64") and len(toks) == 3 and toks[1] == "exec":
            v = f.get(_pair(toks[2]))
            if v is not None:
                f["vcc"] = ("nz" if v == -1 else 0) if op == "s_and_b64" else (0 if v == -1 else "nz")
        return f
    a = _pair(d)
    regs = parse_regs(d)
    for r in [k for k in f if isinstance(k, int) or (isinstance(k, tuple) and k[0] in ("sv", "c"))]:
        x = r if isinstance(r, int) else r[1]  # a write to a tracked register (either half of a pair)
        if ("s", x) in regs or (not (isinstance(r, tuple) and r[0] == "c") and ("s", x + 1) in regs):
            f.pop(r)
    if a is not None and op == "s_mov_b64" and len(toks) == 2:
        t = toks[1]
        if t in ("-1", "0"):
            f[a] = int(t)
        elif _pair(t) is not None and _pair(t) in f:
            f[a] = f[_pair(t)]
    return f


def check_kernel(body: list, name: str, verbose: int = 5, exec_rule: bool = False) -> list:
    """Path-sensitive in the scalar flags (flags_step): a block's entry states
    are kept per flag assignment and joined only within one.  exec_rule: also
    apply the exec-masked row-load rule (module docstring) -- the kernels built
    to it (the 128-wide fused ones); the hand-pipelined kernels keep exec-masked
    loads by design (role branches, masked descriptor loads) and are checked
    for their wait counts only."""
    lines = []
    for l in body:
        l = l.split(";")[0].strip()
        lines.append(l)
    blocks, succ = build_cfg(lines)
    label_block = {lines[a][:-1]: i for i, (a, _) in enumerate(blocks) if lines[a].endswith(":")}
    f0 = (("exec", "full"),)  # a workgroup of whole waves starts with every lane on
    ins = {0: {f0: State()}}
    seen = {}
    hazards = {}
    work = [(0, f0)]
    it = 0
    while work:
        it += 1
        if it > 400000:
            raise RuntimeError(f"{name}: no fixed point")
        i, fk = work.pop()
        st = ins[i][fk].copy()
        flags = dict(fk)
        a, b = blocks[i]
        last = ""
        for k in range(a, b):
            l = lines[k]
            if not l or l.startswith(".") or l.endswith(":"):
                continue
            st.line = k
            st = step(st, l, lambda why, ins_, k=k: hazards.setdefault((k, why), ins_), exec_rule)
            flags = flags_step(flags, l)
            last = l
        nxt = list(succ[i])
        op = last.split()[0] if last else ""
        if op in ("s_cbranch_vccz", "s_cbranch_vccnz") and "vcc" in flags:
            taken = (flags["vcc"] == 0) == (op == "s_cbranch_vccz")
            tgt = label_block.get(last.split()[1])
            nxt = [tgt] if taken else [j for j in nxt if j != tgt]
        elif op in ("s_cbranch_execz", "s_cbranch_execnz") and flags.get("exec") == "full":
            tgt = label_block.get(last.split()[1])
            nxt = [tgt] if op == "s_cbranch_execnz" else [j for j in nxt if j != tgt]
        elif op in ("s_cbranch_scc0", "s_cbranch_scc1") and "scc" in flags:
            tgt = label_block.get(last.split()[1])
            nxt = [tgt] if flags["scc"] == (op == "s_cbranch_scc1") else [j for j in nxt if j != tgt]
        fk2 = tuple(sorted(flags.items(), key=str))
        for j in nxt:
            cur = ins.setdefault(j, {})
            new = st if fk2 not in cur else cur[fk2].join(st)
            kk = new.key()
            if seen.get((j, fk2)) != kk:
                seen[(j, fk2)] = kk
                cur[fk2] = new
                work.append((j, fk2))
    out = sorted(hazards.items())
    for (k, why), ins_ in out[:verbose]:
        print(f"  HAZARD line {k}: {why}: {ins_}")
    print(f"{name} hazards {len(out)}")
    return out


def kernels(asm: str, patterns: list):
    for name in re.findall(r"^(_Z\w+):", asm, re.M):
        if not patterns or any(p in name for p in patterns):
            i = asm.index(name + ":")
            j = asm.index(".Lfunc_end", i)
            yield name, asm[i:j].split("\n")


def main():
    asm = open(sys.argv[1]).read()
    total = 0
    for name, body in kernels(asm, sys.argv[2:]):
        total += len(check_kernel(body, name))
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()


def witness(body: list, load_line: int, use_line: int, max_states: int = 400000):
    """A path (block labels / start lines) from the load at load_line to
    use_line along which no wait retires it, with the same scalar-flag branch
    pruning as check_kernel (for reading a reported hazard)."""
    lines = [l.split(";")[0].strip() for l in body]
    blocks, succ = build_cfg(lines)
    label_block = {lines[a][:-1]: i for i, (a, _) in enumerate(blocks) if lines[a].endswith(":")}
    blk = {}
    for i, (a, b) in enumerate(blocks):
        for k in range(a, b):
            blk[k] = i
    is_ds = lines[load_line].startswith("ds_")
    # flags at the load: taken from any path reaching it (rerun the analysis up to it)
    def run(i, k0, y, flags):
        a, b = blocks[i]
        last = ""
        for k in range(max(a, k0), b):
            l = lines[k]
            if not l or l.startswith(".") or l.endswith(":"):
                continue
            if k == use_line:
                return "hit", y, flags, l
            op = l.split()[0]
            kind = classify(op, l)
            if kind == "wait":
                m = re.search(r"lgkmcnt\((\d+)\)" if is_ds else r"vmcnt\((\d+)\)", l)
                if m and y >= int(m.group(1)):
                    return "retired", y, flags, l
            elif (not is_ds and kind.startswith("vmem")) or (is_ds and kind.startswith("ds_")):
                y = min(y + 1, CAP)
            flags = flags_step(flags, l)
            last = l
        return "open", y, flags, last

    def nexts(i, flags, last):
        nxt = list(succ[i])
        op = last.split()[0] if last else ""
        if op in ("s_cbranch_vccz", "s_cbranch_vccnz") and "vcc" in flags:
            taken = (flags["vcc"] == 0) == (op == "s_cbranch_vccz")
            tgt = label_block.get(last.split()[1])
            nxt = [tgt] if taken else [j for j in nxt if j != tgt]
        elif op in ("s_cbranch_execz", "s_cbranch_execnz") and flags.get("exec") == "full":
            tgt = label_block.get(last.split()[1])
            nxt = [tgt] if op == "s_cbranch_execnz" else [j for j in nxt if j != tgt]
        elif op in ("s_cbranch_scc0", "s_cbranch_scc1") and "scc" in flags:
            tgt = label_block.get(last.split()[1])
            nxt = [tgt] if flags["scc"] == (op == "s_cbranch_scc1") else [j for j in nxt if j != tgt]
        return nxt

    start = blk[load_line]
    frontier = [(start, load_line + 1, 0, {}, (blocks[start][0],))]
    seen = set()
    while frontier and len(seen) < max_states:
        i, k0, y, flags, path = frontier.pop(0)
        r, y2, f2, last = run(i, k0, y, dict(flags))
        if r == "hit":
            return [lines[p] if lines[p].endswith(":") else p for p in path]
        if r == "retired":
            continue
        for j in nexts(i, f2, last):
            key = (j, y2, tuple(sorted(f2.items(), key=str)))
            if key not in seen:
                seen.add(key)
                frontier.append((j, 0, y2, f2, path + (blocks[j][0],)))
    return None
