# gemm_tn: stores vs no stores, and de-phased epilogues (odd workgroups start half / a quarter of a
# tile late) at the N = 1 shapes and the tp2 ring-chunk shapes.
set -u
O=gpurun_out/r5_gemm_skew; mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python benchmarks/bench_gemm_tn.py --only fc1_fwd fc2_fwd qkv_fwd proj_fwd --ablate 8 64 1024 > $O/n1.log 2>&1 && \
timeout -k 10 300 python benchmarks/bench_gemm_tn.py --m 16384 --only fc1_chunk qkv_chunk --ablate 8 64 1024 > $O/chunk.log 2>&1 && \
timeout -k 10 300 python benchmarks/bench_gemm_tn.py --only fc1_fwd fc2_fwd qkv_fwd proj_fwd fc1_dgrad fc2_dgrad qkv_dgrad > $O/ab.log 2>&1
rc=$?; grep -v amdgpu $O/n1.log $O/chunk.log | grep -v '^.*{' ; grep -v amdgpu $O/ab.log | grep -v '{'; exit $rc
