set -e
PROBE_BUFS=4 timeout -k 10 150 ./quic-test_amd/lib/probe_runs 1000000 7 0.01 > gpurun_out/runs_c5d.txt 2>&1
PROBE_BUFS=3 timeout -k 10 150 ./quic-test_amd/lib/probe_runs 1000000 5 0 > gpurun_out/runs_c3d.txt 2>&1
for m in resident coalescer pageable nolaunch; do timeout -k 10 60 ./quic-test_amd/lib/exit_path_test $m 300 >> gpurun_out/exit_path.jsonl 2>>gpurun_out/exit_path.err; echo "rc=$?" >> gpurun_out/exit_path.jsonl; done
grep -v "^check" gpurun_out/runs_c5d.txt gpurun_out/runs_c3d.txt; cat gpurun_out/exit_path.jsonl
timeout -k 10 120 ./quic-test_amd/lib/probe_c4 1000000 7 > gpurun_out/probe_c4.txt 2>&1; cat gpurun_out/probe_c4.txt
