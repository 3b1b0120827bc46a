# Probe: rocpd schema with --marker-trace (kernel + marker trace only)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/mp
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/mp/raw -o bench -- python3 bench.py --steps 20 --no-north-star --no-config3 --no-lsd --no-superpoint --no-cpu-baseline > gpurun_out/mp/bench.json 2>gpurun_out/mp/bench.err
python3 - <<'PY' > gpurun_out/mp/schema.txt
import sqlite3, glob
p = glob.glob("gpurun_out/mp/raw/**/*.db", recursive=True)[0]
c = sqlite3.connect(p)
print(p)
for (n, sql) in c.execute("select name, sql from sqlite_master where type in ('table','view')"):
    print("==", n); print(sql)
for v in ("regions", "region", "markers", "kernels"):
    try:
        cur = c.execute(f"select * from {v} limit 3")
        print("##", v, [d[0] for d in cur.description]); print(cur.fetchall())
    except Exception as e:
        print("##", v, "ERR", e)
PY
rm -rf gpurun_out/mp/raw
