/* tools/sim/spec_sim.c — schedule model (dev tool, not product): per-pixel visit counts of
 * the merged fused schedule with and without speculative sample starts, on the CPU
 * restatement's exact paths (GI).  Built by tools/sim/spec_sim.py. */
#include "../../oracle/oracle.c"

/* integrate_gi with per-trace event recording: for every Scene::intersect of the sample,
 * whether it was predictable before tracing (the path ends after it whatever it hits) and
 * whether the "surface hit" prediction held. */
static v3 integrate_gi_ev(const scene_ctx* C, v3 ro, v3 rd, uint32_t max_depth, orc_mt* rng, path_counters* pc,
                          int* last_pred, int* last_ok) {
    const xrt_scene_desc* S = C->S;
    v3 radiance = mk(0, 0, 0), thr = mk(1, 1, 1);
    uint32_t depth = 0;
    *last_pred = 0, *last_ok = 0;
    while (depth < max_depth) {
        hinfo info;
        hinfo_init(&info);
        pc->segments++;
        int rr_term = 0;
        if (depth > 0) {
            orc_mt peek = *rng;
            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
            rr_term = orc_draw(&peek) >= p;
        }
        const int pred = depth + 1 == max_depth || rr_term;
        const int hit = scene_intersect(S, ro, rd, &info, &pc->tri_tests);
        *last_pred = pred;
        *last_ok = pred && hit && (rr_term || (S->objects[info.hit].light < 0 && S->objects[info.hit].material == XRT_MAT_LAMBERT));
        if (!hit) break;
        if (depth > 0) {
            const float p = smin((thr.x + thr.y + thr.z) / 3.0f, 1.0f);
            if (orc_draw(rng) >= p) break;
            thr = vdivv(thr, mk(p, p, p));
        }
        const xrt_object* ob = &S->objects[info.hit];
        if (ob->light >= 0) {
            if (depth == 0) radiance = vadd(radiance, vmul(thr, light_Le(&S->lights[ob->light], info.ns, rd)));
            break;
        }
        for (uint32_t li = 0; li < S->n_lights; ++li) {
            v3 wi = mk(0, 0, 0);
            float tmax = 0.0f, pdf = 0.0f;
            (void)light_sample(&S->lights[li], info.pos, &wi, &pdf, &tmax, rng);
        }
        float pdf = 1.0f;
        v3 nextDir = mk(0, 0, 0), fr = mk(0, 0, 0);
        if (ob->material == XRT_MAT_LAMBERT) {
            nextDir = lambert_sample_dir(info.ng, info.dpdu, info.dpdv, rng, &pdf);
            fr = eval_bxdf(ob);
        }
        float cosv = smax(.0f, vdot(nextDir, info.ng));
        thr = vmul(thr, vdivs(vmuls(fr, cosv), pdf));
        ro = vadd(info.pos, vmuls(info.ng, 0.01f));
        rd = nextDir;
        depth++;
    }
    return radiance;
}

/* visits[q*3+0]: chain length today (one trace per visit), [q*3+1]: with speculation on a
 * predicted surface hit, [q*3+2]: with every possible next start enumerated */
int sim_visits(const xrt_scene_desc* S, const orc_camera* cam, const xrt_render_params* p, const uint32_t* pi,
               const uint32_t* pj, uint32_t n, uint32_t* visits) {
    scene_ctx C;
    setup_ctx(&C, S, NULL);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t q = 0; q < (int64_t)n; ++q) {
        orc_mt rng;
        orc_mt_seed(&rng, pj[q] + p->width * pi[q]);
        path_counters pc = {0, 0, 0, 0, 0};
        uint32_t spec_saved = 0, enum_visits = 0, unspec = 1;
        for (uint32_t k = 0; k < p->spp; ++k) {
            const float u = ((float)(int)pj[q] + orc_draw(&rng)) / (float)p->width;
            const float v = ((float)(int)pi[q] + orc_draw(&rng)) / (float)p->height;
            v3 ro, rd;
            camera_ray(cam, u, v, &ro, &rd);
            int lp, lok;
            const uint64_t seg0 = pc.segments;
            (void)integrate_gi_ev(&C, ro, rd, p->max_depth, &rng, &pc, &lp, &lok);
            if (lok && k + 1 < p->spp) spec_saved++;
            /* enumerated speculation: every possible next-sample start of a sample's last trace
             * ({c, c+1, c+5}) traced with it and its bounce 0 shaded in the same visit; a start
             * after a sample that ended at its camera ray is traced on its own visit */
            const uint32_t segs = (uint32_t)(pc.segments - seg0);
            enum_visits += segs - 1 + unspec;
            unspec = segs == 1;
        }
        visits[q * 3] = (uint32_t)pc.segments;
        visits[q * 3 + 1] = (uint32_t)pc.segments - spec_saved;
        visits[q * 3 + 2] = enum_visits;
    }
    return 0;
}
