# Can the host write VRAM directly, and what does a host->VRAM->device->host ping-pong cost?
# Kinds in order of risk, each in its own process under a time limit; the first failure ends the
# script (a kind the host cannot touch faults on the host side, before its kernel is launched).
set -e
P=./quic-test_amd/lib/probe_vram_host
timeout -k 5 30 $P host
timeout -k 5 30 $P finegrained
timeout -k 5 30 $P finegrained_direct
timeout -k 5 30 $P uncached_direct
