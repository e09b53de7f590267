#!/bin/bash
# Trial-level throughput of the thesis sweep on ONE GPU (BASELINE.json config 5): the 18-job grid of
# sweeps/experiment_synthetic.sh (3 models x 3 losses x 2 trainers) through the gpu_pool launcher with k trials
# packed per device, reduced data / epochs so a sweep takes minutes.  Per k: sweep wall time, summed trained
# windows and aggregate windows/s over the wall (scripts/sweep_summary.py -> $OUT/sweep.jsonl).
#   OUT=<subdir of gpurun_out>  KS="1 2 4 8"  NS=<datamodule.n_samples>  EPOCHS=<trainer.max_epochs>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-sweep}
mkdir -p $OUT
export TMPDIR=/tmp
for k in ${KS:-1 2 4 8}; do
  d=$OUT/k$k
  rm -rf $d
  t0=$(date +%s.%N)
  timeout -k 10 ${SWEEP_TIMEOUT:-900} bash sweeps/experiment_synthetic.sh hydra/launcher=gpu_pool \
    'hydra.launcher.devices=[0]' hydra.launcher.jobs_per_device=$k hydra.sweep.dir=$d \
    datamodule.n_samples=${NS:-30000} trainer.max_epochs=${EPOCHS:-2} trainer.enable_progress_bar=false \
    > $OUT/k$k.log 2>&1
  rc=$?
  t1=$(date +%s.%N)
  python scripts/sweep_summary.py $d $k $t0 $t1 $rc >> $OUT/sweep.jsonl
  echo "[sweep] k=$k rc=$rc" | tee -a $OUT/status.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
