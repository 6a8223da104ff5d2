set -e
PROBE_SLOTS_POLICY=1 PROBE_BUFS=6 timeout -k 10 200 ./quic-test_amd/lib/probe_runs 1000000 5 0 > gpurun_out/slots_policy_a.txt 2>&1
grep -v "^check" gpurun_out/slots_policy_a.txt
