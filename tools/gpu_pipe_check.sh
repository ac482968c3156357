# bench: default (N=1, sequential) and the N>1 pipelined schedule under a world-1 RCCL group
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-frames 0 --no-secondary > gpurun_out/pipe_seq.json 2> gpurun_out/pipe_seq.err || { echo SEQFAIL; tail gpurun_out/pipe_seq.err; exit 1; }
DMF_BENCH_PIPELINE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --cpu-frames 0 --no-secondary > gpurun_out/pipe_pipe.json 2> gpurun_out/pipe_pipe.err || { echo PIPEFAIL; tail gpurun_out/pipe_pipe.err; exit 2; }
echo ALLOK
