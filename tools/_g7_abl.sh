for abl in 0 1 2 4; do
  UNET_WG_ABL=$abl timeout -k 10 150 python bench.py --dtype bf16 --extra-dtypes= --no-cpu-baseline --no-iou --no-extras --steps 5 --warmup 2 > gpurun_out/g7/abl$abl.json || exit 2
done
