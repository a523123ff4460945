#!/bin/bash
# join ablation: output base atomic removed (noatomic), output stores removed (nostore)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_alt.sh r05m_a "C3 REF-B" noatomic 2 && bash tools/ab_alt.sh r05m_s "C3 REF-B" nostore 2
