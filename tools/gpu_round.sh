#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench (with extra configs), an in-process A/B against a
# reference build, and the config-2 profile (trace + PMC).  Every GPU step has its own time limit;
# the script stops at the first step that faults, aborts or times out (a plain test failure goes on).
# Usage: bash tools/gpu_round.sh <tag> [steps...]
#   steps: probe copyab r6tests pp6 stests policy snapdev rtests tests smoke bench ab prof pp prof3 exp_res res_trace ahead barreq align
#          r4tests abrealign snapab profsnap gtests ftests hostsizes smallwl smalltrace copytrace
#          (default: tests smoke bench ab prof)
set -u
TAG=$1; shift
STEPS=${*:-"tests smoke bench ab prof"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
check() {  # name rc
  echo "$1 rc=$2" | tee -a $OUT/steps.txt
  if [ "$2" -ge 124 ]; then echo "stopping after $1 (rc $2)" | tee -a $OUT/steps.txt; exit "$2"; fi
}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
      check tests $? ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      check smoke $? ;;
    bench)
      timeout -k 10 600 python3 bench.py > $OUT/bench_line.json 2> $OUT/bench.err
      check bench $? ;;
    benchdrv)  # the driver's round-end arguments (BENCH_r05: --steps 20 --warmup 5)
      timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_drv_line.json 2> $OUT/bench_drv.err
      check benchdrv $? ;;
    ab)
      timeout -k 10 300 python3 tools/ab_libs.py ablib/libqgcm_r2.so quantum_amd/libqgcm.so --rounds 15 > $OUT/ab.txt 2>&1
      check ab $? ;;
    spin)  # resident callers allowed to spin at once (QGCM_RESIDENT_SPINNERS; default half the CPU share)
      for rep in 1 2; do
        for sp in 8 12 16; do
          QGCM_RESIDENT_SPINNERS=$sp timeout -k 10 60 tools/bin/per_packet_bench 16 1350 2 0 resident >> $OUT/spin_$sp.jsonl 2>> $OUT/spin.err
          check spin_$sp $?
        done
      done ;;
    ab8)  # config 2 in-process A/B against the build in ${ABLIB:-ablib/flat8}
      timeout -k 10 300 python3 tools/ab_libs.py ${ABLIB:-ablib/flat8}/libqgcm.so quantum_amd/libqgcm.so --rounds 9 > $OUT/ab8.txt 2>&1
      check ab8 $? ;;
    prof)
      bash tools/profile.sh $TAG > $OUT/profile.log 2>&1
      check prof $?
      mkdir -p profiles/$TAG
      python3 tools/trace_summary.py gpurun_out/prof_$TAG > $OUT/kernel_stats_summary.txt 2>&1
      python3 tools/pmc_traffic.py gpurun_out/prof_$TAG 1048576 1350 1408 1048576 > $OUT/traffic_print.txt 2>&1
      cp gpurun_out/prof_$TAG/traffic.json $OUT/ 2>/dev/null ;;
    pp)
      for t in 1 16 64 256; do
        timeout -k 10 120 tools/bin/per_packet_bench $t 1350 2 0 >> $OUT/per_packet.jsonl 2>> $OUT/per_packet.err
        check pp_$t $?
      done
      for t in 16 64; do
        timeout -k 10 120 tools/bin/per_packet_bench $t 1350 2 1 >> $OUT/per_packet.jsonl 2>> $OUT/per_packet.err
        check pp_bulk_$t $?
      done ;;
    stests)
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_snappy.py -x -v --timeout 120 --timeout-method thread > $OUT/snappy_tests.txt 2>&1
      check stests $? ;;
    policy)
      timeout -k 10 400 python3 tools/exp_chain_policy.py 3 > $OUT/chain_policy.jsonl 2> $OUT/chain_policy.err
      check policy $? ;;
    chunks)
      timeout -k 10 500 python3 tools/exp_chain_policy.py 3 chunks > $OUT/chain_chunks.jsonl 2> $OUT/chain_chunks.err
      check chunks $? ;;
    ctests)
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k chain -x -v --timeout 120 --timeout-method thread > $OUT/chain_tests.txt 2>&1
      check ctests $? ;;
    slots)
      timeout -k 10 500 python3 tools/exp_chain_policy.py 3 slots > $OUT/chain_slots.jsonl 2> $OUT/chain_slots.err
      check slots $? ;;
    snapdev)
      timeout -k 10 200 python3 tools/exp_snappy_dev.py 5 > $OUT/snappy_dev.json 2> $OUT/snappy_dev.err
      check snapdev $? ;;
    snapmix)  # the codec's time by data shape (random, one repeated line, config 5, zeros)
      timeout -k 10 200 python3 tools/exp_snappy_mix.py 5 > $OUT/snappy_mix.jsonl 2> $OUT/snappy_mix.err
      check snapmix $? ;;
    profsnap)
      timeout -k 10 900 bash tools/profile_snappy.sh $TAG > $OUT/profile_snappy.log 2>&1
      check profsnap $? ;;
    rtests)
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > $OUT/resident_tests.txt 2>&1
      check rtests $? ;;
    prof3)
      bash tools/profile_config3.sh $TAG > $OUT/profile3.log 2>&1
      check prof3 $? ;;
    exp_res)
      timeout -k 10 600 bash tools/exp_resident.sh $TAG
      check exp_res $? ;;
    res_trace)
      timeout -k 10 300 bash tools/res_trace.sh $TAG
      check res_trace $? ;;
    c5trace)
      bash tools/trace_config5.sh $TAG
      check c5trace $? ;;
    exp_chain)
      timeout -k 10 900 bash tools/exp_chain.sh $TAG
      check exp_chain $? ;;
    barreq)
      timeout -k 10 400 bash tools/exp_barreq.sh $TAG
      check barreq $? ;;
    ahead)  # keystream ahead on / off, interleaved: lone caller and 16 threads (per_packet_bench)
      for rep in 1 2; do
        for a in 1 0; do
          for t in 1 16; do
            QGCM_RESIDENT_AHEAD=$a timeout -k 10 60 tools/bin/per_packet_bench $t 1350 2 0 resident >> $OUT/ahead_$a.jsonl 2>> $OUT/ahead.err
            check ahead_${a}_$t $?
          done
        done
      done ;;
    poll)  # resident kernel A/B against the build in ${ABLIB:-ablib/poll_old} (LD_LIBRARY_PATH comes before RUNPATH)
      for rep in 1 2; do
        for lib in old new; do
          for t in 1 16; do
            if [ $lib = old ]; then
              LD_LIBRARY_PATH=$PWD/${ABLIB:-ablib/poll_old} timeout -k 10 60 tools/bin/per_packet_bench $t 1350 2 0 resident >> $OUT/poll_$lib.jsonl 2>> $OUT/poll.err
            else
              timeout -k 10 60 tools/bin/per_packet_bench $t 1350 2 0 resident >> $OUT/poll_$lib.jsonl 2>> $OUT/poll.err
            fi
            check poll_${lib}_$t $?
          done
        done
      done ;;
    align)  # config 3 packed vs 64-B aligned payloads: time, then WRITE_SIZE / FETCH_SIZE per layout
      timeout -k 10 300 python3 tools/exp_config3_align.py 9 > $OUT/align.json 2> $OUT/align.err
      check align $?
      for form in packed aligned; do
        for c in WRITE_SIZE FETCH_SIZE; do
          timeout -k 10 300 rocprofv3 --pmc $c -d $OUT/pmc_${form}_$c -o $c --output-format csv -- python3 tools/exp_config3_align.py 2 $form > $OUT/pmc_${form}_$c.log 2>&1
          check pmc_${form}_$c $?
        done
        mkdir -p $OUT/pmc_$form && cp -r $OUT/pmc_${form}_*/* $OUT/pmc_$form/ 2>/dev/null
        python3 tools/pmc_config3.py $OUT/pmc_$form > $OUT/traffic_$form.txt 2>&1
      done ;;
    r4tests)  # the suites round 4 changed
      timeout -k 10 900 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_config5.py tests/test_gpu_snappy.py tests/test_bench_dist.py tests/test_gpu_resident.py -x -v --timeout 300 --timeout-method thread > $OUT/r4_tests.txt 2>&1
      check r4tests $? ;;
    profsnap2)  # device snappy counters, four-packets-per-wave encoder and one wave per packet
      for g in 1 0; do  # (exp_snappy_dev alternates the encoders itself; pmc_kernels splits them by name)
        QGCM_SNAPPY_GROUP=$g bash tools/profile_snappy.sh ${TAG}_g$g > $OUT/profsnap_g$g.log 2>&1
        check profsnap_g$g $?
        python3 tools/pmc_kernels.py gpurun_out/prof_snappy_${TAG}_g$g 1048576 snappy_compress snappy_uncompress > $OUT/snappy_pmc_g$g.txt 2>&1
      done ;;
    hostlegs)  # the PCIe-inclusive bench legs, each in a fresh process, with the NUMA nodes of their pinned arenas
      timeout -k 10 600 python3 tools/exp_host_legs.py > $OUT/host_legs.jsonl 2> $OUT/host_legs.err
      check hostlegs $? ;;
    dmaab)  # keyed host batch (DMA runs): staging slots (3 is the default), each in a fresh process
      for sl in ${DMASLOTS:-3 4}; do
        QGCM_GROUP_DMA_SLOTS=$sl timeout -k 10 400 python3 tools/exp_host_legs.py config3_host > $OUT/dmaab_slots$sl.jsonl 2>> $OUT/dmaab.err
        check dmaab_slots$sl $?
      done ;;
    dmachunk)  # keyed host batch (DMA runs): chunk size (per-chunk descriptor-batch cost vs pipeline fill/drain)
      for v in ${DMACHUNKS:-64 256 384 512 768}; do
        QGCM_GROUP_DMA_CHUNK_MB=$v timeout -k 10 400 python3 tools/exp_host_legs.py config3_host > $OUT/dmachunk_$v.jsonl 2>> $OUT/dmachunk.err
        check dmachunk_$v $?
      done ;;
    dmatl)  # keyed host batch: per-chunk GPU timeline from timing events (no profiler), at the chunk sizes in DMACHUNKS x slots in DMASLOTS
      for v in ${DMACHUNKS:-512 768}; do
        for sl in ${DMASLOTS:-4}; do
          q=${HWQ:-4}  # hardware queues per process (HIP's default 4; at most 32 here)
          GPU_MAX_HW_QUEUES=$q QGCM_GROUP_DMA_TIMELINE=1 QGCM_GROUP_DMA_CHUNK_MB=$v QGCM_GROUP_DMA_SLOTS=$sl timeout -k 10 300 python3 tools/run_leg.py config3_host 2 > $OUT/dmatl_${v}_s${sl}_q$q.json 2> $OUT/dmatl_${v}_s${sl}_q$q.err
          check dmatl_${v}_s${sl}_q$q $?
        done
      done ;;
    tracechunk)  # copy / kernel timelines of the keyed host batch at the DMA chunk sizes in TRACECHUNKS
      for v in ${TRACECHUNKS:-512}; do
        QGCM_GROUP_DMA_CHUNK_MB=$v timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_c3_$v -o t -- python3 tools/run_leg.py config3_host 2 > $OUT/trace_c3_$v.log 2>&1
        check tracechunk_$v $?
      done ;;
    legorder)  # does a leg that ran before it slow the pinned-host e2e leg in one process (the bench's order)?
      timeout -k 10 600 python3 tools/exp_host_legs.py e2e config4_one_gpu+e2e config4_one_gpu+sleep30+e2e > $OUT/legorder.jsonl 2> $OUT/legorder.err
      check legorder $? ;;
    gtests)  # the group (multi-GPU drop-in) suite
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_group.py -x -v --timeout 300 --timeout-method thread > $OUT/group_tests.txt 2>&1
      check gtests $? ;;
    copytrace)  # copy / kernel timelines of the keyed host batch and the contiguous pipeline (is H2D overlapping D2H?)
      for leg in config3_host e2e; do
        timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_$leg -o t -- python3 tools/run_leg.py $leg 2 > $OUT/trace_$leg.log 2>&1
        check trace_$leg $?
        python3 tools/copy_trace_summary.py $OUT/trace_$leg > $OUT/copy_summary_$leg.txt 2>&1
      done ;;
    pcieaf)  # PCIe copy rates before and after a 90-GB HBM allocation is freed in the same process
      timeout -k 10 300 python3 tools/microbench/pcie.py --after-free 90 > $OUT/pcie_after_free.jsonl 2> $OUT/pcie_af.err
      check pcieaf $? ;;
    r5tests)  # the suites round 5 changed
      timeout -k 10 900 python3 -u -m pytest tests/test_gpu_group.py tests/test_gpu_parity.py tests/test_cpp_mirror.py tests/test_bench_dist.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r5_tests.txt 2>&1
      check r5tests $? ;;
    crashmaps)  # the exit-time crash under the copy tracer, short form, with the process's maps for resolve_crash.py
      PCIE_MAPS=$OUT/maps_${CRASHTAG:-q}.txt timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_${CRASHTAG:-q} -o t -- python3 tools/microbench/pcie.py --quick ${CRASHARGS:-} > $OUT/trace_${CRASHTAG:-q}.log 2>&1
      rc=$?
      python3 tools/resolve_crash.py $OUT/trace_${CRASHTAG:-q}.log $OUT/maps_${CRASHTAG:-q}.txt > $OUT/resolved_${CRASHTAG:-q}.txt 2>&1
      check crashmaps $rc ;;
    c3traffic)  # config 3's read excess by form (1024 keys vs one key, packed vs 64-B aligned), separate PMC passes
      for form in packed packed_onekey aligned aligned_onekey; do
        i=0
        for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
          i=$((i+1))
          timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/c3t/${form}_p$i -o p --output-format csv -- python3 tools/exp_config3_traffic.py run $form > $OUT/c3t_${form}_p$i.log 2>&1
          check c3t_${form}_p$i $?
        done
      done
      python3 tools/exp_config3_traffic.py summarize $OUT/c3t > $OUT/c3_traffic.json 2>&1 ;;
    crashmin)  # exit-time crash under the copy tracer: which minimal script crashes (steps stop at the first crash)
      for m in ${CRASHMODES:-kernel:kt copy:kt kernel:mc copy_reset:mc copy:mc}; do
        mode=${m%%:*}; tr=${m##*:}
        if [ $tr = kt ]; then TRACE="--kernel-trace"; else TRACE="--kernel-trace --memory-copy-trace"; fi
        timeout -k 10 120 rocprofv3 $TRACE --output-format csv -d $OUT/cm_${mode}_$tr -o t -- python3 tools/microbench/crash_min.py $mode > $OUT/cm_${mode}_$tr.log 2>&1
        rc=$?
        ls -R $OUT/cm_${mode}_$tr 2>/dev/null | grep -c csv > $OUT/cm_${mode}_$tr.csvcount
        check cm_${mode}_$tr $rc
      done ;;
    c3time)  # config 3's four forms timed in one process, interleaved
      timeout -k 10 300 python3 tools/exp_config3_traffic.py time 7 > $OUT/c3_forms_time.json 2> $OUT/c3_forms_time.err
      check c3time $? ;;
    chainpin)  # config 5 from host memory, codec workers pinned per physical core vs left to the scheduler
      timeout -k 10 400 python3 tools/exp_chain_pin.py 2 > $OUT/chain_pin.jsonl 2> $OUT/chain_pin.err
      check chainpin $? ;;
    sntests)  # the snappy / config-5 suites
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_config5.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/sn_tests.txt 2>&1
      check sntests $? ;;
    pcieaftrace)  # the after-free rows under the profiler, kernel trace only: with --memory-copy-trace rocprofv3's own
                  # finalization faults at exit for torch copies on side streams (tools/README.md, crashmin)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_pcieaf -o t -- python3 tools/microbench/pcie.py --after-free 90 > $OUT/trace_pcieaf.log 2>&1
      check pcieaftrace $? ;;
    e2ebig)  # qgcm_seal_host past its 4-GiB staging ring (slots rotate) vs within it
      timeout -k 10 400 python3 tools/exp_host_legs.py e2e e2e_big > $OUT/e2e_big.jsonl 2> $OUT/e2e_big.err
      check e2ebig $? ;;
    members2)  # keyed host batch with two member contexts on this GPU (grouped layout): per-member DMA pipelines side by side, with per-chunk timelines
      for q in ${HWQS:-4}; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python3 tools/exp_host_legs.py config3_host config3_host2 > $OUT/members2_q$q.jsonl 2> $OUT/members2_q$q.err
        check members2_q$q $?
      done ;;
    hostsizes)  # worker-sized host batches: seal+open pair latency and rate vs batch size (qgcm_seal_host and a one-member group)
      timeout -k 10 400 python3 tools/exp_host_batch_sizes.py 30 > $OUT/host_batch_sizes.jsonl 2> $OUT/host_batch_sizes.err
      check hostsizes $? ;;
    smalltrace)  # kernel + copy timeline of 64-packet host and group pairs (where a small call's time goes)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_small -o t -- python3 tools/exp_host_batch_sizes.py 40 64 > $OUT/trace_small.log 2>&1
      check smalltrace $? ;;
    smallwl)  # small keyed batches: worklist in one workgroup vs the multi-launch path, alternating
      timeout -k 10 300 python3 tools/exp_small_worklist.py 30 > $OUT/small_worklist.jsonl 2> $OUT/small_worklist.err
      check smallwl $? ;;
    e2echunk)  # qgcm_seal_host / open_host chunk size (QGCM_PIPE_CHUNK_MB), each in a fresh process
      for v in ${E2ECHUNKS:-32 64 128 256}; do
        QGCM_PIPE_CHUNK_MB=$v timeout -k 10 300 python3 tools/exp_host_legs.py e2e > $OUT/e2echunk_$v.jsonl 2>> $OUT/e2echunk.err
        check e2echunk_$v $?
      done ;;
    ftests)  # the descriptor-batch fuzz and config-3 suites
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_config3.py -x -v --timeout 300 --timeout-method thread > $OUT/fuzz_tests.txt 2>&1
      check ftests $? ;;
    pcie)  # raw pinned-host <-> HBM hipMemcpyAsync rates of this box (the ceiling of every PCIe-inclusive figure)
      timeout -k 10 200 python3 tools/microbench/pcie.py > $OUT/pcie.json 2> $OUT/pcie.err
      check pcie $? ;;
    profsnap3)  # device snappy counters: group encoder (prefetching), wave encoder, decoder
      bash tools/profile_snappy.sh ${TAG}_s3 > $OUT/profsnap3.log 2>&1
      check profsnap3 $?
      python3 tools/pmc_kernels.py gpurun_out/prof_snappy_${TAG}_s3 1048576 snappy_compress_group snappy_compress_kernel snappy_uncompress_kernel > $OUT/snappy_pmc_s3.txt 2>&1 ;;
    probe)  # what GPU telemetry (clock, power, cap) this box gives an unprivileged process
      timeout -k 10 120 python3 tools/probe_telemetry.py > $OUT/telemetry_probe.jsonl 2> $OUT/telemetry_probe.err
      check probe $? ;;
    copyab)  # HBM copy kernel shapes (tools/microbench/copy.hip): the roofline's achievable-copy reference
      for gb in ${COPYGB:-1.48}; do
        timeout -k 10 120 tools/bin/copy_bench $gb 10 > $OUT/copy_bench_$gb.jsonl 2> $OUT/copy_bench.err
        check copyab_$gb $?
      done ;;
    r6tests)  # the suites round 6 changed
      timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tail_pool.py tests/test_cpp_mirror.py tests/test_bench_dist.py tests/test_gpu_snappy.py tests/test_gpu_config5.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r6_tests.txt 2>&1
      check r6tests $? ;;
    pp6)  # per-packet host CPU per pair: resident callers spinning (default) vs all asleep (SPINNERS=0), 16 / 64 threads
      for rep in 1 2; do
        for sp in default 0; do
          for t in 16 64; do
            if [ $sp = default ]; then
              timeout -k 10 60 tools/bin/per_packet_bench $t 1350 2 0 resident >> $OUT/pp6.jsonl 2>> $OUT/pp6.err
            else
              QGCM_RESIDENT_SPINNERS=$sp timeout -k 10 60 tools/bin/per_packet_bench $t 1350 2 0 resident >> $OUT/pp6.jsonl 2>> $OUT/pp6.err
            fi
            check pp6_${sp}_$t $?
          done
        done
      done ;;
    abst)  # steady-state in-process A/B of the working tree's library against the build(s) in ABLIBS
      timeout -k 10 600 python3 tools/ab_steady.py quantum_amd/libqgcm.so ${ABLIBS:-sidelib/pool0/libqgcm.so} --rounds ${ABROUNDS:-5} --steps ${ABSTEPS:-200} --packets ${ABPACKETS:-1048576} > $OUT/ab_steady${ABTAG:-}.jsonl 2> $OUT/ab_steady${ABTAG:-}.err
      check abst $? ;;
    streams)  # the headline step in several stream layouts, interleaved (tools/exp_streams.py)
      timeout -k 10 500 python3 tools/exp_streams.py ${EXP_ROUNDS:-3} 200 > $OUT/streams.jsonl 2> $OUT/streams.err
      check streams $? ;;
    snapocc)  # device snappy encoder time vs the waves per CU it may hold (QGCM_SNAPPY_PER_CU), interleaved
      timeout -k 10 400 python3 tools/exp_snappy_occupancy.py 5 3 > $OUT/snappy_occupancy.jsonl 2> $OUT/snappy_occupancy.err
      check snapocc $? ;;
    snapab)  # device snappy codec: group vs wave encoder, interleaved
      timeout -k 10 300 python3 tools/exp_snappy_dev.py 5 2 > $OUT/snap_ab.jsonl 2> $OUT/snap_ab.err
      check snapab $? ;;
  esac
done
echo all done | tee -a $OUT/steps.txt
