"""Static check of k_riccati_bwd_schur<12,4>'s register staging (kernels_schur.hip):
inside the stage loop, no instruction other than the staging loads and the
LDS writes (lput) may write or read a register of a load set while that set's
loads are in flight.  Reads the assembly of kernels_schur.hip (hipcc -S).
Conservative linear scan over the loop body, wrapping the back edge; prints
the offending lines and exits 1 on a hazard."""
import os
import re
import subprocess
import sys

def regs(op):
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()

# register-staged kernels per source file (kernel name patterns)
KERNELS = {"kernels_schur.hip": r"k_riccati_bwd_schurILi12ELi4E", "kkt_riccati.hip": r"k_kkt_ric_bwdILi"}


def main(src, asm="/tmp/_schur_check.s"):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude",
                           "-mllvm", "-amdgpu-mfma-vgpr-form", "--cuda-device-only", "-S", src, "-o", asm]
                          + os.environ.get("ASM_CHECK_DEFS", "").split(),  # e.g. -DPDPLQR_SCHUR_SPLIT=1 (variants)
                          stderr=subprocess.DEVNULL)
    text = open(asm).read().split("\n")
    pat = KERNELS.get(src.split("/")[-1], KERNELS["kernels_schur.hip"])
    # every compile-time instantiation (L-form and gain-form record, fused penalty; KKT row counts)
    starts = [i for i, l in enumerate(text) if re.match(r"_Z\w*" + pat + r"\w*:", l)]
    if not starts:
        print("no register-staged kernel instantiation found")
        return 1
    rc = 0
    for st in starts:
        end = next(i for i in range(st, len(text)) if text[i].startswith(".Lfunc_end"))
        print(text[st].rstrip(":"))
        body = text[st:end]
        calls = [l.strip() for l in body if l.strip().startswith("s_swappc") or l.strip().startswith("s_setpc")]
        spill = [l for l in stage_loop(body) if l.startswith("scratch_")]
        if calls or spill:  # a call or a spill in the stage loop may move registers with loads in flight
            print("HAZARD: calls / stage-loop scratch traffic in a register-staged kernel:", (calls + spill)[:4])
            rc = 1
        rc |= check(body)
    return rc


def stage_loop(lines):
    """The loop that carries the staging loads (other loops of the kernel, e.g.
    the terminal's penalty rows, are skipped): its instructions."""
    for hdr in (i for i, l in enumerate(lines) if "Loop Header" in l):
        lab = lines[hdr].split(":")[0]
        backs = [i for i, l in enumerate(lines) if re.search(r"s_(c)?branch\w*\s+" + re.escape(lab) + r"\b", l)]
        if not backs:
            continue
        body = lines[hdr:max(backs) + 1]
        ins = [l.strip() for l in body if l.strip() and not l.strip().startswith((";", "."))]
        if any(l.startswith("global_load_dwordx4") for l in ins):
            return ins
    raise SystemExit("no stage loop with staging loads found")


def check(lines):
    ins = stage_loop(lines)
    # in-flight sets: destinations of global_load_dwordx4 in the body
    loads = [(i, regs(l.split()[1].rstrip(","))) for i, l in enumerate(ins) if l.startswith("global_load_dwordx4")]
    bad = []
    L = len(ins)
    for i, r in loads:
        # walk forward (wrapping) until a waitcnt vmcnt that retires this load: we conservatively stop
        # at the first s_waitcnt vmcnt(...) after which ds_write_b128 of these regs happens
        j = (i + 1) % L
        steps = 0
        while steps < L:
            l = ins[j]
            if l.startswith("s_waitcnt") and "vmcnt" in l:
                # the set is consumed after this wait (its ds_write follows); stop at the first wait
                # that precedes a ds_write of r
                k, found = (j + 1) % L, False
                for _ in range(32):
                    if ins[k].startswith("ds_write_b128") and regs(ins[k].split()[2].rstrip(",")) & r:
                        found = True
                        break
                    k = (k + 1) % L
                if found:
                    break
            if not l.startswith("global_load_dwordx4") and not l.startswith("s_"):
                ops = [o.rstrip(",") for o in l.split()[1:]]
                touched = set().union(*[regs(o) for o in ops]) if ops else set()
                if touched & r:
                    bad.append(l)
            j = (j + 1) % L
            steps += 1
    # loop exit: between the last staging load and the exit branch the body must
    # drain the counter (s_waitcnt vmcnt(0)); the exit block may copy or reuse the
    # set registers (the round-1 failure: a copy at the exit, the old registers
    # then reused as MFMA accumulators while the last load was landing)
    last_load = max(i for i, _ in loads)
    exits = [i for i, l in enumerate(ins) if l.startswith("s_cbranch") and i > last_load]
    drained = any(ins[i].startswith("s_waitcnt vmcnt(0)") for i in range(last_load, max(exits) if exits else L))
    if not drained:
        bad.append("loop exit reached with staging loads in flight (no vmcnt(0) after the last load)")
    for b in bad:
        print("HAZARD:", b)
    print(f"loop body {L} instructions, {len(loads)} staging loads, {len(bad)} hazards")
    return 1 if bad else 0

if __name__ == "__main__":
    sys.exit(main(*(sys.argv[1:] or ["pdp-lqr_amd/csrc/kernels_schur.hip"])))
