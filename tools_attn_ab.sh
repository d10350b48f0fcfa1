set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do for v in base prio1 prio2; do
  echo -n "$v r$round: "; MMPFN_LIB=$PWD/multimodalpfn_amd/libmmpfn_var_$v.so timeout -k 10 120 python3 tools_attn_time.py 100 || exit 1
done; done
