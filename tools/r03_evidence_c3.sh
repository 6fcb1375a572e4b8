bash tools/c3_variants.sh "dpp:X=1" "head:X=1:pointcloud_processor_amd/_lib/alt_head/libpcp.so" || exit 1
bash tools/r03_final.sh A
