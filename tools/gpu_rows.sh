source tools/gpu_lib.sh
for r in 1 34 68 135 270 540 1080; do
  ROWS=$r MODES=batch8,batch8_thr run host_rows$r 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2954$((r%10)) tools/host_probe_bands.py || exit 1
done
