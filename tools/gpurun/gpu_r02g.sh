#!/bin/bash
# PMC of quad kernel v2 on WAL verify
R=$(pwd); O=$R/gpurun_out
bash tools/prof_quad.sh r02g_quad || exit $?
python tools/pmc_per_unit.py $O/r02g_quad crc32c_quad_kernel 4352000 --label "WAL verify, quad v2" > $O/r02g_quad/summary.json
head -28 $O/r02g_quad/summary.json
