set -e
mkdir -p gpurun_out/sw
for mh in 224 192 160 128; do
  FRECSYS_DUAL_MAX_H=$mh timeout -k 10 200 python scripts/rank_share.py ials_ml20m_d256 5 8 > gpurun_out/sw/c2_n8_mh$mh.jsonl
  FRECSYS_DUAL_MAX_H=$mh timeout -k 10 200 python scripts/rank_share.py ials_ml20m_d256 5 1 > gpurun_out/sw/c2_n1_mh$mh.jsonl
done
for mh in 256 192; do
  FRECSYS_DUAL_MAX_H=$mh timeout -k 10 300 python scripts/rank_share.py ials_msd_d512 3 8 > gpurun_out/sw/c4_n8_mh$mh.jsonl
done
FRECSYS_S3_PRIO=1 timeout -k 10 200 python scripts/rank_share.py ials_ml20m_d256 5 8 > gpurun_out/sw/c2_n8_s3prio.jsonl
FRECSYS_S3_PRIO=1 timeout -k 10 200 python scripts/rank_share.py ials_ml20m_d256 5 1 > gpurun_out/sw/c2_n1_s3prio.jsonl
FRECSYS_DUAL_PROF=1 timeout -k 10 200 python scripts/rank_share.py ials_ml20m_d256 3 1 > gpurun_out/sw/c2_dualprof.jsonl 2> gpurun_out/sw/c2_dualprof.err
