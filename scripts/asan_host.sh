#!/usr/bin/env bash
# Host-code AddressSanitizer run of the C++ mirror test (batcher, shim, host mirror).
#   bash scripts/asan_host.sh build   # in the build container: instrumented copies in build/asan/
#   bash scripts/asan_host.sh run     # on the GPU box
#   SAN=thread: the same with ThreadSanitizer into build/tsan/ (HIP runtime frames suppressed)
# The shim and batcher are compiled with -Xarch_host -fsanitize=address (device code is not
# instrumented: GPU sanitizers are not available on this pool), the mirror and its test with
# clang++ -fsanitize=address, against the product's kernel object.  Leak checking is off (the
# HIP runtime keeps allocations until exit).  The quarantine is large enough never to recycle
# during the run: ASan's device-memory allocator CHECK-fails when a device chunk parked in the
# quarantine is recycled after the HIP runtime has unloaded at exit (sanitizer_allocator_device.h).
set -euo pipefail
cd "$(dirname "$0")/.."
SANK=${SAN:-address}
A=build/$([ "$SANK" = thread ] && echo tsan || echo asan)
case "${1:-run}" in
  build)
    mkdir -p $A
    H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -fvisibility=hidden -Iinclude -Iquic-test_amd/csrc"
    SANF="-Xarch_host -fsanitize=$SANK -Xarch_host -fno-omit-frame-pointer"
    $H -x hip -c -o $A/fec_shim.o quic-test_amd/csrc/fec_shim.cpp $SANF
    $H -x hip -c -o $A/fec_batcher.o quic-test_amd/csrc/fec_batcher.cpp $SANF
    $H -x hip -c -o $A/fec_coalesce.o quic-test_amd/csrc/fec_coalesce.cpp $SANF
    RT=$([ "$SANK" = thread ] && echo "" || echo -shared-libasan)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fsanitize=$SANK $RT -o $A/libfec_hip.so \
      quic-test_amd/lib/fec_kernels.o quic-test_amd/lib/src_hash.o $A/fec_shim.o $A/fec_batcher.o $A/fec_coalesce.o
    C="/opt/rocm/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=$SANK $RT -fno-omit-frame-pointer -Iinclude -Iquic-test_amd/host"
    $C -fPIC -shared -o $A/libquicfec_host.so quic-test_amd/host/fec.cpp -L$A -lfec_hip -Wl,-rpath,'$ORIGIN'
    $C -o $A/host_mirror_test tests/csrc/host_mirror_test.cpp -L$A -lquicfec_host -lfec_hip oracle/liboracle.so \
      -Wl,-rpath,'$ORIGIN' -Wl,-rpath,'$ORIGIN/../../oracle' -lpthread
    $C -o $A/ctx_isolation_test tests/csrc/ctx_isolation_test.cpp -L$A -lfec_hip -Wl,-rpath,'$ORIGIN' -lpthread
    # the unchanged call site from 16 streams through the resident encoder and shared launches
    $C -o $A/batcher_latency quic-test_amd/csrc/tools/batcher_latency.cpp -Iquic-test_amd/csrc -L$A -lquicfec_host -lfec_hip \
      oracle/liboracle.so -Wl,-rpath,'$ORIGIN' -Wl,-rpath,'$ORIGIN/../../oracle' -lpthread
    # mixed shapes through both resident ring kinds (the VRAM ring's host-side packing and tagged
    # row collection), pageable and page-locked buffers
    $C -rdynamic -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o $A/exit_path_test tests/csrc/exit_path_test.cpp \
      -L$A -lfec_hip -ldl -Wl,-rpath,'$ORIGIN'
    [ "$SANK" = thread ] || cp /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so $A/
    printf 'called_from_lib:libamdhip64.so\ncalled_from_lib:libhsa-runtime64.so\nrace:libamdhip64.so\nrace:libhsa-runtime64.so\n' > $A/tsan.supp
    ;;
  run)
    export LD_LIBRARY_PATH=$A
    export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:verify_asan_link_order=0:halt_on_error=1:quarantine_size_mb=16384
    export TSAN_OPTIONS="suppressions=$A/tsan.supp:report_signal_unsafe=0:second_deadlock_stack=1:history_size=4"
    timeout -k 10 600 $A/host_mirror_test
    timeout -k 10 300 $A/ctx_isolation_test
    QUICFEC_RESIDENT=1 timeout -k 10 120 $A/batcher_latency legacy 16 0 2
    QUICFEC_RESIDENT=0 timeout -k 10 120 $A/batcher_latency legacy 16 0 2
    QUICFEC_RESIDENT_VRAM=0 timeout -k 10 120 $A/batcher_latency legacy 16 0 2
    timeout -k 10 120 $A/exit_path_test mixed 360
    timeout -k 10 120 $A/exit_path_test mixed_hostring 360
    # round 5: the ring's tag hooks (torn chunks, late address words, epoch scrubs) and poisoning
    # under 8 threads, through the same host code
    timeout -k 10 120 $A/exit_path_test tear 300
    timeout -k 10 300 $A/exit_path_test epoch 6144
    timeout -k 10 300 $A/exit_path_test poison_mt 2400
    # relaunch cycles under 4 threads (8 serving classes, the default), and the tag runs with one class
    timeout -k 10 300 $A/exit_path_test cycles_mt 2000
    QUICFEC_RESIDENT_SERVERS=1 timeout -k 10 120 $A/exit_path_test tear 300
    QUICFEC_RESIDENT_SERVERS=1 timeout -k 10 300 $A/exit_path_test poison_mt 2400
    ;;
esac
