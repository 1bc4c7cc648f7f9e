"""The device modules the test suite renders (__graft_entry__.build()
precompiles them next to the product's, pathtrace.modules): the zoo scenes,
the option variants the GPU tests run, pt_trace_rays' ray-list modules, the
query modules and the PT_DEVICE_DEFINES variants.  Test infrastructure: the
product's own list is path-trace_amd/pathtrace/modules.py."""
import os


def test_jobs():
    import pathtrace as pt
    import zoo
    jobs = [((lambda b=b: pt.DeviceScene(zoo.build(b))), d) for (_, b, _, _, _, d) in zoo.RENDER_CASES]
    jobs += [((lambda b=b: pt.DeviceScene(zoo.build(b))), d) for (b, d) in zoo.GPU_ONLY_CASES]
    # tests/test_gpu_parity.py test_fast_spine_bitexact
    jobs += [((lambda b=b: pt.DeviceScene(zoo.build(b), fast_spine=True)), d)
             for (b, d) in [("csg_zoo", 6), ("scene_p1", 8), ("union_zoo", 6)]]
    # tests/test_gpu_parity.py test_lane_walk_bitexact / test_lane_walk_c5_same_bits
    from test_gpu_parity import LANE_WALK_CASES
    jobs += [((lambda b=b, k=k: pt.DeviceScene(zoo.build(b), lane_walk=k)), d) for (b, d, k) in LANE_WALK_CASES]
    # test_lane_scatter_bitexact, test_c2_lane_scatter_same_bits_as_wave, the C2 config-golden tests
    from test_gpu_parity import LANE_SCATTER_CASES
    jobs += [((lambda b=b: pt.DeviceScene(zoo.build(b), lane_scatter=True)), d) for (b, d) in LANE_SCATTER_CASES]
    jobs += [((lambda b=b: pt.DeviceScene(zoo.build(b))), d) for (b, d) in LANE_SCATTER_CASES if b == "scatter_zoo"]
    # tests/test_trace_rays.py: pt_trace_rays' ray-list modules (each scene option it runs)
    from test_trace_rays import CASES as TR_CASES, MODES as TR_MODES
    from test_trace_rays import TEX_CASES as TR_TEX
    tr = {(b, ()) for (_, b) in TR_CASES} | {(b, tuple(sorted(o.items()))) for (_, b, o) in TR_MODES}
    jobs += [(lambda b=b, o=o: _rays(b, dict(o)), None) for (b, o) in sorted(tr)]
    jobs += [(lambda b=b, d=d: pt.DeviceScene(zoo.build(b)).compile_rays(d), None) for (b, d) in TR_TEX]
    # tests/test_queries.py: the boundary's query modules (span lists, texture lookups)
    jobs += [(lambda b=b: _queries(b, None), None) for b in ("csg_zoo", "scene_p1")]
    jobs += [(lambda b=b, k=k: _queries(b, k), None) for b, n in zip(zoo.TEX_EVAL_SCENES, TEX_EVAL_COUNTS)
             for k in range(n)]
    # tests/test_user_texture.py, tests/test_facade.py: user Texture subclasses (pt_tex_device)
    from test_user_texture import user_scene, facade_user_scene, CHECKER_FACADE
    jobs += [((lambda: pt.DeviceScene(user_scene())), 4), ((lambda: pt.DeviceScene(facade_user_scene())), 6),
             ((lambda: pt.DeviceScene(facade_user_scene(CHECKER_FACADE))), 6)]
    # tests/test_user_object.py: user Object subclasses (pt_object_device)
    from test_user_object import p0, box_scene
    jobs += [((lambda: pt.DeviceScene(p0(True))), 6), ((lambda: pt.DeviceScene(p0(False))), 6),
             ((lambda: pt.DeviceScene(box_scene())), 6), ((lambda: pt.DeviceScene(box_scene()).compile_queries()), None)]
    # tests/test_zero_child.py: skies of finite and non-finite emission
    from test_zero_child import CASES as ZC_CASES, SKIES, sky_scene, DEPTH as ZC_DEPTH
    jobs += [((lambda s=s, k=k: pt.DeviceScene(sky_scene(SKIES[s]()), lane_walk=k)), ZC_DEPTH) for (s, k) in ZC_CASES]
    # tests/test_occlude.py: plane occluders near the emitters
    from test_occlude import VARIANTS as OC_VARIANTS, DEPTH as OC_DEPTH
    jobs += [((lambda v=v: pt.DeviceScene(zoo.occlude_box(v))), OC_DEPTH) for v in OC_VARIANTS]
    return jobs


def _rays(builder, opts):
    import pathtrace as pt
    import zoo
    from test_trace_rays import _golden
    depth = _golden("p1" if builder == "scene_p1" else "csg")[3]
    pt.DeviceScene(zoo.build(builder), **opts).compile_rays(depth)
    return None


TEX_EVAL_COUNTS = (36, 20)  # textures of zoo.TEX_EVAL_SCENES (tests/golden/tex_eval.npz)


def _queries(builder, tex):
    import pathtrace as pt
    import zoo
    from pathtrace.scene import to_text
    ds = pt.DeviceScene.from_text(to_text(zoo.build(builder), "/tmp/pt_build_img_%d" % os.getpid()))
    if tex is None:
        ds.compile_queries()
    else:
        pt._lib.check(pt._lib.lib().pt_query_compile(ds.handle, -2, int(tex)))
    return None


# device-library variants the GPU tests compile: (defines, builder, depth, lane_scatter) --
# tests/test_gpu_parity.py test_round_cut_paths_bitexact, test_lane_scatter_run_cap_same_bits
TEST_DEFINES = [("PT_ROOM_CAP=3", "scene_p1", 8, False), ("PT_ROOM_CAP=40", "scene_p1", 8, False),
                ("PT_LANE_RUN_CAP=3", "scatter_zoo", 6, True),
                # test_lds_poison_bitexact (POISON_CASES)
                ("PT_POISON_LDS=1 PT_ROOM_CAP=3", "scene_p1", 8, False),
                ("PT_POISON_LDS=1 PT_ROOM_CAP=3", "csg_zoo", 6, False),
                # test_occlusion_settles_more_children
                ("PT_OCCLUDE=0", "occlude_box", 3, False)]
