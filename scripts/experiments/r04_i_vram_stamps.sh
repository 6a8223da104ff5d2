# Where the VRAM ring's ~30 us a call goes: the server's phase stamps (QUICFEC_RESIDENT_STAMPS)
# for the three inline store forms (4: 12-B chunk columns as three 32-bit stores; 12: one 12-B
# store each; 16: 16-B columns) and the page-locked ring, one stream and 16.  Output: gpurun_out/r04i/.
# (QUICFEC_RESIDENT_INLINE_STORE existed only on the build this ran on; the library kept one form.)
set -e
mkdir -p gpurun_out/r04i
B=./quic-test_amd/lib/batcher_latency
for form in 4 12 16 host; do
  if [ $form = host ]; then e="QUICFEC_RESIDENT_VRAM=0"; else e="QUICFEC_RESIDENT_INLINE_STORE=$form"; fi
  env $e QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy_raw 5000 > gpurun_out/r04i/raw_$form.json 2> gpurun_out/r04i/raw_$form.err || [ $? -eq 1 ]
  env $e QUICFEC_RESIDENT_STAMPS=1 timeout -k 10 60 $B legacy 16 0 1 > gpurun_out/r04i/s16_$form.json 2> gpurun_out/r04i/s16_$form.err || [ $? -eq 1 ]
  echo "== $form"; cat gpurun_out/r04i/raw_$form.json gpurun_out/r04i/raw_$form.err gpurun_out/r04i/s16_$form.json gpurun_out/r04i/s16_$form.err | grep -E "delay_us|resident_stamps" | cut -c1-400
done
