# Headline step vs tile height at 640x480 batch 1 (FD_TILE_H), two rounds.
set -e
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/th
for i in 1 2; do for th in 2 3 4 6; do
  FD_TILE_H=$th timeout -k 10 200 python3 bench.py --steps 300 --no-config3 --no-superpoint --no-lsd --no-cpu-baseline --no-north-star > gpurun_out/th/b.json 2>/dev/null
  python3 -c "import json;d=json.load(open('gpurun_out/th/b.json'));print('tile_h $th', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
