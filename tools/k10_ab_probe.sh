# K10 A/B of abvar/base.so vs abvar/new.so at the four SuperPoint layer shapes and the whole forward
set -e
cd $GRAFT_REPO_ROOT
for L in base new base new; do
  for ly in conv1b conv2a conv2b conv3a; do
    FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 60 python3 tools/sp_k10_probe.py --layer $ly --calls 10 | sed "s/^/$L /"
  done
  FD_LIB_PATH=$GRAFT_REPO_ROOT/abvar/$L.so timeout -k 10 120 python3 tools/sp_forward_time.py
done
