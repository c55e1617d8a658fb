#!/bin/bash
# the drop forms A/B: kernel stats of tools/sparse_codec_run.py with the emit form (default) and the
# image form (ONO_DROP_FORM=image), then sp_phases of both
# usage: tools/emit_ab.sh TAG
set -e
T=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in emit image; do
    ONO_DROP_FORM=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/${T}_$f -o p -- python3 tools/sparse_codec_run.py 10 > gpurun_out/${T}_$f.log 2>&1
    echo "== $f"; grep "^drop" gpurun_out/${T}_$f.log
    python3 tools/kstats.py gpurun_out/${T}_$f | grep -E "sp_|thresh" || true
    ONO_DROP_FORM=$f timeout -k 10 60 tools/sp_phases 64 24 > gpurun_out/${T}_phases_$f.txt 2>&1
    grep -E "^# sp_ph|units" gpurun_out/${T}_phases_$f.txt
done
