#!/bin/bash
# Build libewk.so from a git revision (or the working tree with "WT") into variants/<name>.so,
# optionally with extra -D flags:  scripts/build_variant.sh <rev|WT> <name> [-DFOO=1 ...]
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
REV=$1; NAME=$2; shift 2
T=$(mktemp -d)
mkdir -p "$T/easywakeword_amd/csrc" "$T/include" "$R/variants"
SRCS="ewk_mfcc.hip ewk_gate.hip ewk_level3.hip ewk_engine.cpp ewk_tables.cpp"
for f in easywakeword_amd/csrc/ewk_gather.hip; do   # sources that older revisions lack
  if [ "$REV" = "WT" ] || git -C "$R" cat-file -e "$REV:$f" 2>/dev/null; then SRCS="$SRCS $(basename $f)"; fi
done
HDRS="ewk_internal.h ewk_gate.h"
for h in ewk_rescore.h ewk_fp4.h ewk_fp4_mel.h ewk_db64.h; do   # headers that some revisions lack (ewk_fp4*.h: round 5 only)
  if { [ "$REV" = "WT" ] && [ -f "$R/easywakeword_amd/csrc/$h" ]; } || \
     { [ "$REV" != "WT" ] && git -C "$R" cat-file -e "$REV:easywakeword_amd/csrc/$h" 2>/dev/null; }; then HDRS="$HDRS $h"; fi
done
for s in $SRCS $HDRS; do
  f=easywakeword_amd/csrc/$s
  if [ "$REV" = "WT" ]; then cp "$R/$f" "$T/$f"; else git -C "$R" show "$REV:$f" > "$T/$f"; fi
done
if [ "$REV" = "WT" ]; then cp "$R/include/ewk.h" "$T/include/ewk.h"; else git -C "$R" show "$REV:include/ewk.h" > "$T/include/ewk.h"; fi
objs=""
for s in $SRCS; do
  x=""; [ "$s" = ewk_mfcc.hip ] && x="-fno-slp-vectorize"   # as easywakeword_amd/build.py EXTRA
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function $x "$@" \
     -c "$T/easywakeword_amd/csrc/$s" -o "$T/$s.o" &
  objs="$objs $T/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/variants/$NAME.so" $objs
rm -rf "$T"
echo "$R/variants/$NAME.so"
