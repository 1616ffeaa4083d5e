import shutil, subprocess, sys, pathlib
R = pathlib.Path('/root/repo')
VAR = {
 'v5': [("      kw1 = x1 >= 0 ? (int)klist[x1] : 0;\n    };", "      kw1 = x1 >= 0 ? (int)klist[x1] : 0;\n      __builtin_amdgcn_s_waitcnt(0xC07F);\n    };")],
 'v1': [("      if (retire) {\n        // tile T0's diagonal position", "      if (false && retire) {\n        // tile T0's diagonal position")],
 'v2': [("      v[s] = x < prm.t_cut ? 0.0 : e;", "      v[s] = e;")],
 'v3': [("      if (i2 >= cend) continue;                              // (wave-uniform)\n      if (i2 < n_act) {", "      if (true) continue;\n      if (i2 < n_act) {"),
        ("    if (tid < PT) {\n      const int ns = cend - c0;", "    if (false) {\n      const int ns = cend - c0;")],
 'v4': [("      return o < 64 ? __builtin_amdgcn_readlane(kw0, o) : __builtin_amdgcn_readlane(kw1, o - 64);", "      return x + 0 * o;")],
}
for v, pats in VAR.items():
    if len(sys.argv) > 1 and v not in sys.argv[1:]: continue
    d = R / 'tools' / f'ab_{v}'
    shutil.rmtree(d, ignore_errors=True)
    d.mkdir(parents=True)
    shutil.copytree(R / 'gpmdm_amd', d / 'gpmdm_amd', ignore=shutil.ignore_patterns('_build', '__pycache__', '*.so'))
    shutil.copytree(R / 'include', d / 'include')
    shutil.copy(R / 'bench.py', d / 'bench.py')
    f = d / 'gpmdm_amd' / 'csrc' / 'obs_cutoff.h'
    s = f.read_text()
    for a, b in pats:
        assert a in s, (v, a[:40])
        s = s.replace(a, b)
    f.write_text(s)
    r = subprocess.run([sys.executable, '-m', 'gpmdm_amd.build'], cwd=d, capture_output=True, text=True)
    print(v, r.returncode, r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:])
