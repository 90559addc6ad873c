"""The C-ABI without Python (VERDICT r2 missing #2, SURVEY.md 8b `ewk_gather_detections`):
examples/c_positives_rccl scores K batches through libewk.so, compacts each batch's
positives on the device with `ewk_compact_positives` (append mode) and gathers the records
with RCCL (all_gather of the counts, then the records to rank 0), as INTEGRATION.md section 4
shows; it checks rank 0's records against the scorer's own match/score outputs.  World size
1 here (one MI355X); the binary is built by __graft_entry__.build()."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "c_positives_rccl")
WAV = os.path.join(ROOT, "tests", "golden", "reference_word.wav")


@pytest.mark.parametrize("n_seg,steps", [(4096, 3), (1, 2), (20001, 1)])
def test_c_host_compacts_and_gathers_positives(n_seg, steps):
    if not os.path.exists(BIN):   # optional example: build() warns when hipcc/RCCL cannot build it
        pytest.skip("examples/c_positives_rccl not built (see __graft_entry__.build's warning)")
    env = dict(os.environ, RANK="0", WORLD_SIZE="1")
    r = subprocess.run([BIN, WAV, str(n_seg), str(steps)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK"), r.stdout
