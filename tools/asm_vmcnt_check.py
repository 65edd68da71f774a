"""Static check of the inline-asm load pipelines (a development helper).

  hipcc ... --cuda-device-only -S spmm.hip -o /tmp/sp.s
  python tools/asm_vmcnt_check.py /tmp/sp.s [kernel-substring]

spmm_hub_kernel issues its gathers as inline asm with counted vmcnt waits,
so the compiler does not know those registers are still being written.
This walks each matching kernel's ISA, models the in-order vector-memory
queue (s_waitcnt vmcnt(N) retires all but the N newest loads) and reports
any instruction that reads or overwrites a register whose load may still be
in flight -- e.g. a copy the register allocator placed at a loop back edge,
or a temporary given the register of a load whose value is dead.

Control flow: the text is scanned once in order, then every loop body (a
backward branch to an earlier label) is scanned again starting from the
queue state at its back edge, so loop-carried loads are modelled too.
Branches inside a body are treated as fall-through (both sides scanned).
"""

import re
import sys


def regs(tok):
    tok = tok.split()[0] if tok.split() else tok
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def step(line, pend, report):
    """Apply one instruction to the pending-load queue; report hazards."""
    op = line.split()[0]
    args = [a.strip() for a in line[len(op):].split(",")]
    busy = set().union(*pend) if pend else set()
    if op.startswith("s_waitcnt") and "vmcnt" in line:
        n = int(re.search(r"vmcnt\((\d+)\)", line).group(1))
        return pend[len(pend) - n:] if 0 < n < len(pend) else ([] if n == 0 else pend)
    if op.startswith(("global_load", "scratch_load", "buffer_load")):
        srcs = set().union(*[regs(a) for a in args[1:]])
        if srcs & busy:
            report("address reads an in-flight register", line)
        if regs(args[0]) & busy:
            report("load into an in-flight destination", line)
        return pend + [regs(args[0])]
    srcs = set().union(*[regs(a) for a in args[1:]]) if len(args) > 1 else set()
    if op.startswith("v_pk_") and "op_sel_hi:[1,0]" in line and len(args) > 2:
        srcs = regs(args[1]) | {min(regs(args[2]) or {-1})}  # src1 high lane takes its low half
    dst = regs(args[0]) if args else set()
    if op.startswith(("global_store", "ds_write", "buffer_store", "scratch_store")):
        srcs |= dst
    elif dst & busy:
        report("overwrite of an in-flight destination", line)
    if srcs & busy:
        report("read of an in-flight register", line)
    return pend


def check(body, name):
    lines = [l.split(";")[0].strip() for l in body]
    labels = {l[:-1]: k for k, l in enumerate(lines) if l.startswith(".LBB") and l.endswith(":")}
    hazards = []
    states = {}

    def scan(lo, hi, pend, tag):
        for k in range(lo, hi):
            l = lines[k]
            states[k] = pend
            if not l or l.startswith(".") or l.endswith(":"):
                continue
            pend = step(l, pend, lambda why, ins: hazards.append((tag, k, why, ins)))
        return pend

    scan(0, len(lines), [], "linear")
    for k, l in enumerate(lines):
        m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < k:
            top = labels[m.group(2)]
            scan(top, k + 1, states.get(k, []), f"loop {m.group(2)}")
    for tag, k, why, ins in hazards[:5]:
        print(f"  HAZARD [{tag}] line {k}: {why}: {ins}")
    print(name, "hazards", len(hazards))
    return len(hazards)


def main():
    s = open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/sp.s").read()
    pat = sys.argv[2] if len(sys.argv) > 2 else "spmm_hub_kernel"
    total = 0
    for name in [n for n in re.findall(r"^(_Z\w+):", s, re.M) if pat in n]:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        total += check(s[i:j].split("\n"), name)
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
