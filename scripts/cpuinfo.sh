set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
g++ -O3 -march=x86-64-v3 -o /tmp/scb scripts/microbench/shuffle_chain_bench.cpp && timeout 120 /tmp/scb > gpurun_out/chain_v3.txt 2>&1
g++ -O3 -march=x86-64-v4 -o /tmp/scb4 scripts/microbench/shuffle_chain_bench.cpp && timeout 120 /tmp/scb4 > gpurun_out/chain_v4.txt 2>&1
g++ -O3 -march=native -o /tmp/scbn scripts/microbench/shuffle_chain_bench.cpp && timeout 120 /tmp/scbn > gpurun_out/chain_native.txt 2>&1
head -50 gpurun_out/chain_*.txt
