set -o pipefail
o=gpurun_out/g10
mkdir -p $o
timeout -k 10 900 python bench.py --retune --tune-db-out $o/tune_db.txt --tuning-report $o/tuning.txt > $o/bench.json || exit 3
bash tools/ablate.sh $o/wf $o/tune_db.txt fp32 "UNET_WF64_ABL=0" "UNET_WF64_ABL=1" "UNET_WF64_ABL=2" "UNET_WF64_ABL=4" "UNET_WF64_ABL=8" "UNET_WF64_ABL=6" || exit 4
bash tools/ablate.sh $o/mp $o/tune_db.txt bf16 "UNET_MPB_BLOCKS=1024" "UNET_MPB_CONTIG=1" "UNET_MPB_BLOCKS=4096 UNET_MPB_CONTIG=1" "UNET_MPB_BLOCKS=512 UNET_MPB_CONTIG=1" "UNET_WG_ABL=0" || exit 5
