for i in 1 2; do for v in old new; do
  if [ $v = old ]; then L=$PWD/easywakeword_amd/_var/libewk_old.so; else L=$PWD/easywakeword_amd/libewk.so; fi
  EWK_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 2 --no-cpu-baseline --fixed-len 0 --short-len 0 --confirm-batch 0 --no-host-ingest --max-streams 0 --big-ticks 100 > gpurun_out/ab_${v}_$i.log 2>&1 || exit 1
  echo "$v $i: $(python scripts/stream_line.py gpurun_out/ab_${v}_$i.log | tr '\n' ' ')"
done; done
