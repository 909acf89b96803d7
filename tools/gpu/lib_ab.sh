# Same-box A/B of libvtseg variants (tools/exp/lib_<name>.so; "cur" = the
# in-tree library) on one video: env_ab.py's timing (RUNS decodes after a
# warm-up, stage times, result digest) per variant, PASSES alternating passes.
#   bash tools/gpu/lib_ab.sh VIDEO RUNS OUT_DIR name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
VIDEO=$1; RUNS=$2; O=$3; shift 3
mkdir -p $O
LIB=video-transformer_amd/vtseg/libvtseg.so
cp $LIB /tmp/lib_intree.so
for pass in $(seq ${PASSES:-2}); do
  for v in "$@"; do
    if [ "$v" = cur ]; then cp /tmp/lib_intree.so $LIB; else cp tools/exp/lib_$v.so $LIB; fi
    timeout -k 10 300 python tools/gpu/env_ab.py $VIDEO $RUNS $v= > $O/lib_${v}_$pass.json 2> $O/lib_${v}_$pass.err || { tail -20 $O/lib_${v}_$pass.err; cp /tmp/lib_intree.so $LIB; exit 1; }
    cat $O/lib_${v}_$pass.json
  done
done
cp /tmp/lib_intree.so $LIB
