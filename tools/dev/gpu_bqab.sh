mkdir -p gpurun_out/bqab gpurun_out/shard
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bqab/all.log 2>&1 || { tail -20 gpurun_out/bqab/all.log; exit 1; }
tail -1 gpurun_out/bqab/all.log
XM_AUDIO_LIB=$PWD/xm-audio-utils_amd/lib_ab/libxm_audio.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "biquad or effects or eq or c4 or multi or stream or fir" > gpurun_out/bqab/t.log 2>&1 || { tail -20 gpurun_out/bqab/t.log; exit 1; }
tail -1 gpurun_out/bqab/t.log
for i in 1 2; do for v in A B; do L=xm-audio-utils_amd/lib/libxm_audio.so; [ $v = B ] && L=xm-audio-utils_amd/lib_ab/libxm_audio.so; XM_AUDIO_LIB=$PWD/$L timeout -k 10 200 python3 -u tools/bench_configs.py bq fir --fir-k 15,63 > gpurun_out/bqab/$v$i.log 2>&1 || exit 1; echo $v $(grep -o "\"ms_per_step\": [0-9.]*\|parity_check\": [a-z]*" gpurun_out/bqab/$v$i.log); done; done
for gc in 4096 2048 1024 512; do timeout -k 10 200 python3 -u bench.py --global-clips $gc --steps 20 --warmup 5 --no-cpu > gpurun_out/shard/g$gc.log 2>&1 || exit 1; echo $gc $(grep -o "\"ms_per_step\": [0-9.]*\|\"avg_launch_ms\": [0-9.]*\|\"parity_check\": [a-z]*" gpurun_out/shard/g$gc.log); done
