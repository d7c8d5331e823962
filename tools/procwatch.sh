# diagnostic: what processes does bench.py leave or spawn (run on the GPU box)
python bench.py --steps 3 --warmup 1 --cpu-seconds 1 > gpurun_out/pw_bench.log 2>&1 &
B=$!
sleep 12
ps -eo pid,ppid,pgid,stat,etime,comm,args --forest > gpurun_out/pw_during.txt
wait $B; echo "bench rc $?" >> gpurun_out/pw_during.txt
sleep 1
ps -eo pid,ppid,pgid,stat,etime,comm,args --forest > gpurun_out/pw_after.txt
