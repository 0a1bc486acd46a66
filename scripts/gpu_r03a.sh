#!/bin/bash
# round 3, first GPU check: IPC probe (two processes, one GPU), then the GPU test suite
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f /tmp/ipcp.s /tmp/ipcp.c
timeout -k 10 60 ./tools/ipc_probe_bin server /tmp/ipcp > gpurun_out/ipc_server.log 2>&1 &
P1=$!
sleep 1
timeout -k 10 60 ./tools/ipc_probe_bin client /tmp/ipcp > gpurun_out/ipc_client.log 2>&1
R2=$?
wait $P1
R1=$?
echo "ipc probe rc server=$R1 client=$R2"
cat gpurun_out/ipc_server.log gpurun_out/ipc_client.log
for r in $R1 $R2; do
  if [ $r -ge 124 ]; then echo "probe timed out / crashed: stopping"; exit 1; fi
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_r03a.log 2>&1
R=$?
tail -5 gpurun_out/gputest_r03a.log
exit $R
