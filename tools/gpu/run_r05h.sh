# Round 5 debug: h264_recon_sched on the tiny stream with kernel printf
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h
mkdir -p $O
cp tools/exp/lib_${V:-rsdbg}.so video-transformer_amd/vtseg/libvtseg.so
VTS_RECON_SCHED=1 timeout -k 5 60 python -u tools/debug/rs_tiny.py /tmp/tiny.mp4 > $O/tiny_${V:-rsdbg}.log 2>&1
rc=$?
echo "rc=$rc"
tail -5 $O/tiny_${V:-rsdbg}.log
exit $rc
