#!/bin/bash
# PMC of the span kernel on 16 Mi x 4 KiB descriptors (tools/prof_desc.sh)
set -o pipefail
bash tools/prof_desc.sh
