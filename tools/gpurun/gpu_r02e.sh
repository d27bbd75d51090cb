#!/bin/bash
# PMC of the quad kernel on WAL verify
R=$(pwd); O=$R/gpurun_out
bash tools/prof_quad.sh r02e_quad || exit $?
python tools/pmc_per_unit.py $O/r02e_quad crc32c_quad_kernel 4352000 --label "WAL verify, quad v1" > $O/r02e_quad/summary.json
cat $O/r02e_quad/summary.json
