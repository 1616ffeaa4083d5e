for spec in "cholinv 12000"; do
  set -- $spec
  timeout -k 10 100 python -u tools/trsm_probe.py $1 $2 2>&1 | grep -E "ok|Error" | cut -c1-150
done
echo "--- with ROCBLAS_DEVICE_MEMORY_SIZE=8GiB"
ROCBLAS_DEVICE_MEMORY_SIZE=8589934592 timeout -k 10 100 python -u tools/trsm_probe.py trsm 20000 2>&1 | grep -E "ok|Error" | cut -c1-150
exit 0
