"""pm_config_load against the reference's own TOML parser.

oracle/_ref/toml_check is our driver compiled against the reference's vendored
toml11 4.2.0 (common/src/toml.hpp, where it lies; recipe oracle/ref/Makefile).
It reads every key the reference's two mains read, with the reference's
accessors. For each config variant, our loader must agree key by key:
same values, an error where toml11's accessor throws on a present key of the
wrong type, "absent" where the key is missing, and failure on a syntax error.
Skipped where the reference checkout was not available to build the driver."""
import os
import subprocess

import numpy as np
import pytest

import conftest

TOML_CHECK = os.path.join(conftest.ROOT, "oracle", "_ref", "toml_check")
pytestmark = pytest.mark.skipif(not os.access(TOML_CHECK, os.X_OK),
                                reason="oracle/_ref/toml_check not built (needs the reference checkout)")

BASE = open(os.path.join(conftest.GOLDEN, "config.toml.example")).read()
VARIANTS = {
    "example": BASE,
    "exp_float": BASE.replace("fovy = 0.87", "fovy = 8.7e-1"),
    "hex_int": BASE.replace("max_depth = 10", "max_depth = 0xA"),
    "oct_bin_int": BASE.replace("samples_per_pixel = 24", "samples_per_pixel = 0o30").replace(
        "depth = 30", "depth = 0b1_1110"),
    "plus_int": BASE.replace("max_depth = 10", "max_depth = +10"),
    "literal_str": BASE.replace('"result.png"', "'res\\ult.png'"),
    "escape_str": BASE.replace('"result.png"', '"a\\tb\\u0041\\U0001F600.png"'),
    "ml_array": BASE.replace("fb_size = [800, 600]", "fb_size = [\n  800, # w\n  600,\n]"),
    "inf_float": BASE.replace("fovy = 0.87", "fovy = -inf"),
    "int_for_float": BASE.replace("fovy = 0.87", "fovy = 1"),
    "int_in_vec3": BASE.replace("look_up = [0.0, 1.0, 0.0]", "look_up = [0, 1.0, 0.0]"),
    "float_for_int": BASE.replace("depth = 30", "depth = 30.0"),
    "missing_key": BASE.replace("depth = 30\n", ""),
    "missing_table": BASE.replace("[photon-mapper]", "[photon-mapper-x]"),
    "bad_syntax": BASE.replace("depth = 30", "depth = = 30"),
    "dotted_key": BASE.replace("[photon-mapper]\nmax_depth = 10", "[photon-mapper]\nmax_depth = 10\nx.y = 1"),
    "dotted_table": BASE.replace("[ray-tracer]", "[ray-tracer]\n[dummy.inner]\nq = 1\n[ray-tracer]")
    .replace("[ray-tracer]\n[dummy.inner]\nq = 1\n[ray-tracer]", "[dummy.inner]\nq = 1\n\n[ray-tracer]"),
    "underscore": BASE.replace("1_000", "1_000_000"),
    "comments": BASE.replace("fovy = 0.87", "fovy = 0.87 # field of view\n# trailing comment"),
}
KEYS = ["camera.look_from", "camera.look_at", "camera.look_up", "camera.fovy", "data.photons_file",
        "data.caustics_photons_file", "data.model_path", "ray-tracer.sky_colour", "ray-tracer.output_filename",
        "ray-tracer.fb_size", "ray-tracer.samples_per_pixel", "ray-tracer.depth", "photon-mapper.max_depth",
        "photon-mapper.casted_diffuse_photons", "photon-mapper.casted_caustics_photons"]


def _ours(cfg, key):
    import pm_amd
    if not pm_amd.config_key_present(cfg, key):
        return None
    f3 = lambda v: [np.float32(v.x), np.float32(v.y), np.float32(v.z)]
    return {
        "camera.look_from": lambda: f3(cfg.look_from), "camera.look_at": lambda: f3(cfg.look_at),
        "camera.look_up": lambda: f3(cfg.look_up), "camera.fovy": lambda: [np.float32(cfg.fovy)],
        "data.photons_file": lambda: cfg.photons_file.decode(),
        "data.caustics_photons_file": lambda: cfg.caustics_photons_file.decode(),
        "data.model_path": lambda: cfg.model_path.decode(),
        "ray-tracer.sky_colour": lambda: f3(cfg.sky_colour),
        "ray-tracer.output_filename": lambda: cfg.output_filename.decode(),
        "ray-tracer.fb_size": lambda: [cfg.fb_width, cfg.fb_height],
        "ray-tracer.samples_per_pixel": lambda: [cfg.samples_per_pixel], "ray-tracer.depth": lambda: [cfg.depth],
        "photon-mapper.max_depth": lambda: [cfg.max_depth],
        "photon-mapper.casted_diffuse_photons": lambda: [cfg.casted_diffuse_photons],
        "photon-mapper.casted_caustics_photons": lambda: [cfg.casted_caustics_photons],
    }[key]()


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_config_matches_toml11(name, tmp_path):
    import pm_amd
    path = tmp_path / "config.toml"
    path.write_bytes(VARIANTS[name].encode())
    ref_lines = subprocess.run([TOML_CHECK, str(path)], capture_output=True, check=True).stdout.decode()
    ref_lines = ref_lines.splitlines()
    try:
        cfg = pm_amd.load_config(str(path))
        err = None
    except pm_amd.PMError as e:
        cfg, err = None, str(e)
    if ref_lines == ["PARSE_ERROR"]:
        assert err is not None, "toml11 rejects the file, pm_config_load accepted it"
        return
    ref = {}
    for line in ref_lines:
        key, _, rest = line.partition(" ")
        ref[key] = rest
    wrong_type = [k for k in KEYS if ref[k] == "ERR" and k.split(".")[-1] in VARIANTS[name]
                  and f"[{k.split('.')[0]}]" in VARIANTS[name] and not name.startswith("missing")]
    if wrong_type:
        # toml11's accessor throws on a present key of the wrong type: we refuse the file
        assert err is not None and any(k in err for k in wrong_type), (wrong_type, err)
        return
    assert err is None, err
    for k in KEYS:
        mine = _ours(cfg, k)
        if ref[k] == "ERR":
            assert mine is None, (k, mine)
            continue
        if k in ("data.photons_file", "data.caustics_photons_file", "data.model_path", "ray-tracer.output_filename"):
            assert mine == ref[k], (k, mine, ref[k])
        elif k in ("ray-tracer.fb_size", "ray-tracer.samples_per_pixel", "ray-tracer.depth") or \
                k.startswith("photon-mapper."):
            assert mine == [int(x) for x in ref[k].split()], (k, mine, ref[k])
        else:
            exp = [np.float32(float(x)) for x in ref[k].split()]
            assert [float(a) for a in mine] == [float(b) for b in exp], (k, mine, exp)
