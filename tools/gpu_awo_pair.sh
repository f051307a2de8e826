export YALM_LIB=$PWD/yalm_amd/ab/libyalm_hip_wt_ab.so
for dt in fp16 fp8; do for c in 30 1000 4090; do for pr in 0 1; do
  echo "== $dt ctx $c pair $pr"
  YALM_AWO_PAIR=$pr timeout -k 10 120 python -u tools/attn_wo_trace.py --ctx $c --dtype $dt --time 200 2>&1 | grep -E "launch span|head signalled|Wo slice|Wo poll passed|P.V in LDS|time_kernel" || exit 1
done; done; done
