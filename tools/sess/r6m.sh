# T5 1-doc: LM-head weight loads non-temporal (keep the decoder working set in the MALL?)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
ABN=lmnt_t5 ROUNDS=3 T=300 CMD="python -u bench/summarize.py --docs 1 --steps 20 --warmup 3" A="ATPU_LM_NT=0" B="ATPU_LM_NT=1" CUT=250 bash tools/ab.sh
