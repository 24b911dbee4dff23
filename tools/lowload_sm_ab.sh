mkdir -p gpurun_out
for sm in 256 1024; do
  LOWLOAD_SIZES=256,512,1024 LOWLOAD_SMALL_MAX=$sm LOWLOAD_NREQ=512 timeout -k 10 300 python -u tools/lowload_probe.py > gpurun_out/ll_sm$sm.json 2> gpurun_out/ll_sm$sm.err || { tail -5 gpurun_out/ll_sm$sm.err; exit 1; }
done
