# Profile session: kernel-trace stats + separate PMC passes for cars and
# unicycle (k=3) at B=65536, summarised into small files; raw rocprofv3
# output is deleted on the box (gpurun copies back at most 64 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1
OUT=gpurun_out/$TAG
bash scripts/gpu_session.sh $TAG prof profu pmcf pmcw pmcfu pmcwu pmcv || exit $?
f() { find "$1" -name "$2" | sort | sed -n 1p; }
python scripts/pmc_traffic.py "$(f $OUT/pmc_fetch '*counter_collection.csv')" "$(f $OUT/pmc_write '*counter_collection.csv')" "k_safe_step<0, 0, 1>" $OUT/pmc_traffic_cars_B65536.json env=SimulatedCars B=65536 || exit 1
python scripts/pmc_traffic.py "$(f $OUT/pmc_fetch_u '*counter_collection.csv')" "$(f $OUT/pmc_write_u '*counter_collection.csv')" "k_safe_step<0, 1, 3>" $OUT/pmc_traffic_unicycle3_B65536.json env=Unicycle k=3 B=65536 || exit 1
python scripts/pmc_sq.py "$(f $OUT/pmc_valu '*counter_collection.csv')" "k_safe_step<0, 0, 1>" > $OUT/pmc_sq_cars_B65536.txt || exit 1
cp "$(f $OUT/prof '*kernel_stats.csv')" $OUT/cars_B65536_kernel_stats.csv || exit 1
cp "$(f $OUT/profu '*kernel_stats.csv')" $OUT/unicycle3_B65536_kernel_stats.csv || exit 1
rm -rf $OUT/prof $OUT/profu $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_fetch_u $OUT/pmc_write_u $OUT/pmc_valu
