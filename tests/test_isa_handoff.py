"""The cross-workgroup hand-offs of the fp64 re-score launches, checked in the gfx950 ISA (CPU).

MI355X_MICROARCH.md ("Compiler hazard"): ROCm 7.2 drops the `s_waitcnt vmcnt(0)` after a
release's `buffer_wbl2` when the wave's scoreboard looks empty, so a flag or counter can
overtake the L2 write-back.  Round 5's k_rescore_ring / k_rescore_linear had exactly that
(`buffer_wbl2 sc1; buffer_inv sc1; global_atomic_add`): the last workgroup's poll-mirror copy
could read a re-scored event's float32 score.  This compiles csrc/ewk_mfcc.hip to gfx950
assembly and checks, in every re-score kernel, that each L2 write-back is followed by a vmcnt
wait before the next atomic or store, and each invalidate by a vmcnt wait before the kernel
reads on (ewk_rescore.h score_tail / tick_end)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "easywakeword_amd", "csrc", "ewk_mfcc.hip")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not present")
    out = tmp_path_factory.mktemp("isa") / "ewk_mfcc.s"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "--cuda-device-only",
                    "-S", SRC, "-o", str(out)], check=True, capture_output=True)
    return out.read_text()


def _kernel(asm: str, name_part: str) -> list:
    names = re.findall(r"^\s*\.type\s+(\S+),@function", asm, re.M)
    bodies = []
    for n in names:
        if name_part in n:
            i = asm.index(n + ":")
            j = asm.index(".Lfunc_end", i)
            bodies.append([l.strip() for l in asm[i:j].split("\n")])
    return bodies


def _instrs(body):
    return [l for l in body if l and not l.startswith((";", ".", "/")) and not l.endswith(":")]


@pytest.mark.parametrize("kernel", ["k_rescore_ring", "k_rescore_linear"])
def test_release_waits_before_count_and_acquire_waits_before_loads(asm, kernel):
    bodies = _kernel(asm, kernel)
    assert bodies, kernel
    n_wb = 0
    for body in bodies:
        ins = _instrs(body)
        for k, l in enumerate(ins):
            if l.startswith("buffer_wbl2"):
                n_wb += 1
                nxt = ins[k + 1:k + 4]
                # a vmcnt(0) wait must come before any atomic / store / load that follows
                for m in nxt:
                    if m.startswith("s_waitcnt") and "vmcnt(0)" in m:
                        break
                    assert not re.match(r"(global|flat|buffer)_(atomic|store|load)", m), (kernel, ins[k:k + 4])
            if l.startswith("buffer_inv"):
                nxt = ins[k + 1:k + 3]
                ok = any(m.startswith("s_waitcnt") and "vmcnt(0)" in m for m in nxt) or \
                    any(m.startswith("s_endpgm") for m in nxt)
                assert ok, (kernel, ins[k - 1:k + 3])
    assert n_wb >= 1
