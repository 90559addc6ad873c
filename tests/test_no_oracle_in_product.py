"""The product package never imports or calls the oracle (CPU)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_product_does_not_reference_oracle():
    pkg = os.path.join(ROOT, "easywakeword_amd")
    offenders = []
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                if re.search(r"^\s*(from|import)\s+oracle\b|oracle\.|mfcc_ref|gate_ref", txt, re.M):
                    offenders.append(f)
    assert not offenders, offenders
