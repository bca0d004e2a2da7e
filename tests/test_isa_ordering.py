"""The cross-XCD hand-offs, pinned in the emitted gfx950 ISA.

Two places pass data between workgroups that may sit on different XCDs, whose L2s are not
coherent with each other (MI355X_MICROARCH.md, "inter-workgroup visibility"):

- the planner's decoupled look-back (csrc/spmm_plan.h): a block stores its totals / prefix, then
  its status word; a successor polls the status word, then reads the totals / prefix;
- the in-kernel hub reduce (hub_tail, csrc/spmm_csr_impl.h, every Cfg::LR configuration): a chunk
  stores its partial row, then counts itself in with an atomic add; the last arrival reads every
  partial row.

Neither uses a release/acquire pair (each costs an L2 write-back / invalidate); correctness rests on
the measured gfx950 form (the guide's hand-off table, row 1): every payload store `sc1`, an
`s_waitcnt vmcnt(0)` after the stores and before the signal, and every payload load `sc1`, issued
only after the signal's value has returned.  This test reads that order off `make asm` (the fp32
and bf16 instantiation units and the backward unit) so that a compiler change that moved or
dropped any of it fails here, not in a race on the hardware.  `make asm-ab-handoff` builds the same
units with the order removed (OFX_AB_UNORDERED_HANDOFF); with OFX_ISA_AB=1 the test asserts that
this build is rejected (profiles/r05_isa_ordering_ab.txt records that run).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "of-spmm_amd")
UNITS = ("spmm_inst_f32_i32.s", "spmm_inst_bf16_i32.s", "spmm_backward.s")

VMEM_STORE = re.compile(r"^(global|buffer|flat)_store\w*\s")
VMEM_LOAD = re.compile(r"^(global|buffer|flat)_load\w*\s")
ATOMIC_ADD = re.compile(r"^global_atomic_add\s")
WAIT_VM0 = re.compile(r"^s_waitcnt\s+(.*\b)?vmcnt\(0\)")


def has_sc1(ins):
    return re.search(r"\bsc1\b", ins) is not None


def functions(path):
    """{mangled name: [instruction, ...]} of the kernels in one .s file (comments and directives
    dropped; labels kept as 'LABEL <name>'; inline-asm markers kept as 'ASMSTART' / 'ASMEND')."""
    out, name, body = {}, None, []
    with open(path) as f:
        for raw in f:
            line = raw.rstrip("\n")
            m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
            if m:
                name, body = m.group(1), []
                continue
            if name is None:
                continue
            if line.startswith(".Lfunc_end"):
                out[name] = body
                name = None
                continue
            s = line.strip()
            if s.startswith(";;#ASMSTART"):
                body.append("ASMSTART")
            elif s.startswith(";;#ASMEND"):
                body.append("ASMEND")
            elif re.match(r"^\.?LBB\S*:", s):
                body.append("LABEL " + s)
            elif s and not s.startswith((";", ".")):
                body.append(s.split(";")[0].strip())
    return out


def demangled(name):
    try:
        return subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
    except OSError:
        return name


def check_planner(ins):
    """Publishing: each wait_stores() (the inline `s_waitcnt vmcnt(0)`) sits between sc1 payload
    stores and the sc1 status store.  Polling: payload loads are sc1 and follow a vmcnt(0) that
    comes after the last poll; no plain load reads look words."""
    errs = []
    publishes = 0
    for i, x in enumerate(ins):
        if x != "ASMSTART" or i + 2 >= len(ins) or not WAIT_VM0.match(ins[i + 1]) or ins[i + 2] != "ASMEND":
            continue
        nxt = next((y for y in ins[i + 3:] if VMEM_STORE.match(y) or VMEM_LOAD.match(y) or ATOMIC_ADD.match(y)), None)
        prv = next((y for y in reversed(ins[:i]) if VMEM_STORE.match(y) or VMEM_LOAD.match(y)), None)
        if nxt is not None and VMEM_STORE.match(nxt):
            publishes += 1
            if not has_sc1(nxt):
                errs.append(f"status store after the store wait is not sc1: {nxt}")
            if prv is None or not (VMEM_STORE.match(prv) and has_sc1(prv)):
                errs.append(f"the store wait does not follow sc1 payload stores: {prv}")
    if publishes < 2:
        errs.append(f"{publishes} status publishes behind an inline store wait (expected the totals "
                    f"and the inclusive prefix)")
    # polls: sc1 loads followed by a vmcnt(0) wait within a few instructions, inside a sleep loop
    # (round 5: the statuses of up to four windows are polled together, each load behind its own
    # exec mask, the wait after the last, the sleep after the checks)
    loads = [(i, x) for i, x in enumerate(ins) if VMEM_LOAD.match(x)]
    sc1_loads = [(i, x) for i, x in loads if has_sc1(x)]
    if not sc1_loads:
        return errs + ["no sc1 load in the look-back"]
    sleep = [i for i, x in enumerate(ins) if x.startswith("s_sleep")]
    polls = [i for i, x in sc1_loads if any(WAIT_VM0.match(y) for y in ins[i + 1:i + 8])
             and any(0 < s - i < 48 for s in sleep)]
    if not polls:
        return errs + ["no status poll (sc1 load + vmcnt(0) inside the sleep loop)"]
    first, last_poll = min(polls), max(polls)
    payload = [(i, x) for i, x in sc1_loads if i > last_poll]
    if len(payload) < 4:
        errs.append(f"{len(payload)} sc1 payload loads after the poll (expected the totals / prefix)")
    for i, x in payload:
        if not any(WAIT_VM0.match(y) for y in ins[last_poll + 1:i]):
            errs.append(f"payload load issued before the polled status returned: {x}")
    end = max(i for i, _ in payload) if payload else last_poll
    plain = [x for i, x in loads if first <= i <= end and not has_sc1(x)]
    if plain:
        errs.append(f"plain loads inside the look-back (read through L1): {plain[:3]}")
    return errs


def check_hub_tail(ins):
    """Each arrival count (global_atomic_add, value returned) comes after an s_waitcnt vmcnt(0)
    that follows the partial row's sc1 stores; the partial rows are read with sc1 loads issued
    after the count has returned."""
    errs = []
    adds = [i for i, x in enumerate(ins) if ATOMIC_ADD.match(x)]
    for a in adds:
        stores = [j for j in range(a) if VMEM_STORE.match(ins[j])]
        if not stores:
            errs.append("arrival count with no store before it")
            continue
        last = stores[-1]
        if not has_sc1(ins[last]):
            errs.append(f"the store before the arrival count is not sc1: {ins[last]}")
        if not any(WAIT_VM0.match(y) for y in ins[last + 1:a]):
            errs.append(f"no s_waitcnt vmcnt(0) between the partial store and the arrival count "
                        f"({ins[last]} ... {ins[a]})")
        if " sc0" not in ins[a] and not ins[a].endswith("sc0"):
            errs.append(f"arrival count does not return its value: {ins[a]}")
        later = [j for j in range(a + 1, len(ins)) if VMEM_LOAD.match(ins[j])]
        if not later:
            errs.append("no partial-row load after the arrival count")
            continue
        if not any(WAIT_VM0.match(y) for y in ins[a + 1:later[0]]):
            errs.append(f"a load issued before the arrival count returned: {ins[later[0]]}")
        if not any(has_sc1(ins[j]) for j in later):
            errs.append("partial rows read without sc1 loads")
    return errs


def scan(asm_dir):
    report, planners, tails = [], 0, 0
    for unit in UNITS:
        path = os.path.join(asm_dir, unit)
        for name, ins in functions(path).items():
            if "spmm_plan_kernel" in name:
                planners += 1
                report += [f"{unit} {demangled(name)[:90]}: {e}" for e in check_planner(ins)]
            elif any(ATOMIC_ADD.match(x) for x in ins) and "spmm_main_kernel" in name:
                tails += 1
                report += [f"{unit} {demangled(name)[:90]}: {e}" for e in check_hub_tail(ins)]
    return report, planners, tails


def build_asm(target, build_dir):
    jobs = str(min(os.cpu_count() or 1, 8))
    r = subprocess.run(["make", "-s", "-j", jobs, "-C", PKG, target], capture_output=True, text=True,
                       timeout=1500)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return os.path.join(PKG, build_dir, "asm")


def test_cross_xcd_handoffs_are_ordered_in_the_isa():
    report, planners, tails = scan(build_asm("asm", "build"))
    # every unit has its planner instantiations; the fp32 / bf16 units hold the LR forms
    assert planners >= 6, planners
    assert tails >= 20, tails
    assert not report, "\n".join(report[:40])


@pytest.mark.skipif(os.environ.get("OFX_ISA_AB") != "1",
                    reason="A/B check of the test itself (OFX_ISA_AB=1; ~5 min of device compiles)")
def test_unordered_handoff_build_is_rejected():
    report, planners, tails = scan(build_asm("asm-ab-handoff", "build_ab_handoff"))
    assert planners >= 6 and tails >= 20
    print(f"{len(report)} ordering violations in the unordered build, e.g.:")
    for r in report[:12]:
        print("  " + r)
    assert report, "the A/B build without the hand-off order passed the ordering checks"
