"""Static check of the scorer's inline-asm LDS loads (gfx950 ISA).

The frame pass and the DCT issue their LDS reads as inline asm (`ds_read_b64` / `ds_read_b128`
in EWK_LD64 / EWK_LD128_8 / EWK_DCT_RD) and wait for them with their own asm `s_waitcnt
lgkmcnt(n)`.  The compiler's wait-count pass does not look inside inline asm, and gfx950 has no
hardware interlock on a VGPR whose LDS load is still in flight: if the compiler moves, copies
or otherwise reads (or overwrites) a load's destination register between the asm load and the
asm wait, that instruction sees the register's OLD contents whenever the LDS is slow -- a
silent, load-dependent wrong value.

This walks the assembly of every k_score_f32 instance in program order, keeps the destination
VGPRs of the asm LDS loads that are still outstanding (an asm `s_waitcnt lgkmcnt(n)` retires all
but the newest n of them; LDS returns in order), and reports every non-asm instruction that
reads or writes one of them.  Branches are followed linearly (the loads and their waits sit in
straight-line code).

    python scripts/asm_lds_hazard.py [file.s]     (default: compiles csrc/ewk_mfcc.hip)
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_mfcc.hip")


def vregs(tok):
    """VGPR numbers named by one operand token (v7, v[4:7]); AGPRs / SGPRs ignored."""
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def operands(line):
    body = line.split(";")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])]
    return parts[0], ops


def check(asm_text, kernel_filter="k_score_f32"):
    issues = []
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", asm_text, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if kernel_filter not in name:
            continue
        pending = []        # list of sets (dest VGPRs of outstanding asm LDS loads), oldest first
        in_asm = False
        n_loads = n_waits = 0
        for ln, line in enumerate(body.split("\n")):
            s = line.strip()
            if s.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if s.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
                continue
            op, ops = operands(s)
            if in_asm:
                if op.startswith("ds_read") and ops:
                    pending.append(vregs(ops[0]))
                    n_loads += 1
                elif op == "s_waitcnt":
                    mm = re.search(r"lgkmcnt\((\d+)\)", s)
                    if mm:
                        keep = int(mm.group(1))
                        pending = pending[len(pending) - keep:] if keep else []
                        n_waits += 1
                continue
            if op == "s_waitcnt":
                mm = re.search(r"lgkmcnt\((\d+)\)", s)
                if mm:   # a compiler wait also retires outstanding asm loads
                    keep = int(mm.group(1))
                    pending = pending[len(pending) - keep:] if keep else []
                continue
            if not pending or op.startswith("s_"):
                continue
            live = set().union(*pending)
            touched = set()
            for o in ops:
                touched |= vregs(o)
            hit = touched & live
            if hit:
                issues.append((name, ln, s, sorted(hit)))
        yield name, n_loads, n_waits, issues
        issues = []


def main():
    if len(sys.argv) > 1:
        text = open(sys.argv[1]).read()
    else:
        out = "/tmp/ewk_mfcc_hazard.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                        "--cuda-device-only", "-S", SRC, "-o", out], check=True, capture_output=True)
        text = open(out).read()
    total = 0
    for name, nl, nw, issues in check(text):
        print(f"{name}: {nl} asm LDS loads, {nw} asm waits, {len(issues)} instructions touching an in-flight load's VGPRs")
        for _, ln, s, hit in issues[:20]:
            print(f"    line {ln}: {s}    <- v{hit}")
        total += len(issues)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
