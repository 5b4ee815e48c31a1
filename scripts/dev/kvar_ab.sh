R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python scripts/dev/kvariant.py run base pgs_spec fastdiv pgs_spec_fastdiv base pgs_spec fastdiv pgs_spec_fastdiv || exit 1
HG_LIB=$R/build/kvar/base/libhgsim.so OUT=gpurun_out/a.npz timeout -k 10 200 python scripts/dev/kstep_bits.py run > gpurun_out/bits.log 2>&1 || { tail gpurun_out/bits.log; exit 1; }
HG_LIB=$R/build/kvar/pgs_spec/libhgsim.so OUT=gpurun_out/b.npz timeout -k 10 200 python scripts/dev/kstep_bits.py run >> gpurun_out/bits.log 2>&1 || { tail gpurun_out/bits.log; exit 1; }
python scripts/dev/kstep_bits.py compare gpurun_out/a.npz gpurun_out/b.npz
