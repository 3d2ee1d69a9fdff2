"""A/B of library builds: each build in its own process, interleaved over
rounds (A B C A B C ...), median per build.  Prints the JSON lines and a table.
python scripts/lib_ab.py --libs base,nowrap [--rounds 3] [-- knn_time.py args]
A name resolves to nbodyhpc_amd/lib/exp/<name>/libnbkd.so ("prod" = the
production build); "lib@KNOB=V+..." adds environment knobs (upper case) or
nbkd_set_tuning values (lower case, e.g. prod@self_order=0)."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    libs, rounds = ["prod"], 3
    for j, x in enumerate(argv):
        if x == "--libs":
            libs = argv[j + 1].split(",")
        if x == "--rounds":
            rounds = int(argv[j + 1])
    res = {name: [] for name in libs}
    for r in range(rounds):
        for name in libs:
            env = dict(os.environ)
            # "lib@VAR=V+VAR2=W": a build plus environment knobs (the experiments
            # build, `python -m nbodyhpc_amd.build --experiments`, is "exp")
            lib, _, knobs = name.partition("@")
            tunes = []
            for kv in filter(None, knobs.split("+")):
                kk, _, vv = kv.partition("=")
                if kk.islower():
                    tunes += ["--tune", kv]
                else:
                    env[kk] = vv
            if lib == "exp":
                env["NBKD_LIB"] = os.path.join(ROOT, "nbodyhpc_amd", "lib", "exp", "libnbkd.so")
            elif lib != "prod":
                env["NBKD_LIB"] = os.path.join(ROOT, "nbodyhpc_amd", "lib", "exp", lib, "libnbkd.so")
            out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "knn_time.py")] + extra
                                 + tunes,
                                 env=env, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(out.stdout, out.stderr, flush=True)
                sys.exit(out.returncode)
            line = json.loads(out.stdout.strip().splitlines()[-1])
            line["name"] = name
            print(json.dumps(line), flush=True)
            res[name].append(line)
    print("name                      wall_ms  collect  select  leaf_key  sort  self  retry  sha",
          flush=True)
    for name, ls in res.items():
        med = lambda f: statistics.median(f(x) for x in ls)  # noqa: E731
        if ls[0].get("ball"):
            print(f"{name:24s} {med(lambda x: x['wall_ms']):8.2f}  (radius count) "
                  f"{','.join(sorted(set(x['sha'] for x in ls)))}", flush=True)
            continue
        print(f"{name:24s} {med(lambda x: x['wall_ms']):8.2f} {med(lambda x: x['phases_ms']['knn_collect']):8.2f} "
              f"{med(lambda x: x['phases_ms']['knn_select']):7.2f} {med(lambda x: x['phases_ms']['leaf_key']):8.2f} "
              f"{med(lambda x: x['phases_ms']['sort']):5.2f} "
              f"{med(lambda x: x['phases_ms'].get('self_order', 0.0)):5.2f} "
              f"{med(lambda x: x['phases_ms']['knn_retry']):6.2f} "
              f"{','.join(sorted(set(x['sha'] for x in ls)))}", flush=True)


if __name__ == "__main__":
    main()
