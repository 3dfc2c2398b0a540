#!/bin/bash
# Round 5: the whole GPU suite on the final library, then smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  suite 1100 "python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread" \
  smoke 120 "python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
