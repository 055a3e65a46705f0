for v in head newengine noks ""; do
  MTE_LIB=$v timeout -k 10 100 python tools/sweep.py --docs 1,4096 --modes lds --hw 8 > gpurun_out/v_${v:-cur}.log 2>&1 || exit 1
done
