/*
 * icp_hip.h — C-ABI of libicp_hip.so, the MI355X (gfx950) device path of the ICP
 * correspondence-and-alignment loop. Plain C types only; one context drives one GPU; several
 * contexts (one process per GPU) cooperate through an RCCL communicator.
 *
 * Reference interfaces these entry points replace (B1AnKAlpha/IterativeClosestPoint):
 *   icp_hip_set_target   Octree::Octree(const std::vector<Point3D>&, int max_pts, int max_d)
 *                        PointCloudRegistration/core/octree.h:29, octree.cpp:41-126
 *                        (CLI copy icp_registration.cpp:154-190)
 *   icp_hip_nn           Octree::findNearest(const Point3D&) per query + residual
 *                        octree.h:32, octree.cpp:175-184; icpengine.cpp:172-206
 *   icp_hip_set_source   src/src3d packing, icpengine.cpp:139-152 (CLI :459-470)
 *   icp_hip_iterate      one loop body of ICPEngine::runICP up to the SVD:
 *                        icpengine.cpp:168-337 (NN, residuals, 3-sigma, cull, RMSE, centroids,
 *                        cross-covariance), with the previous iteration's src = T*src
 *                        (icpengine.cpp:345) fused in front. CLI twin: icp_registration.cpp:481-585
 *   icp_hip_apply        src = T * src (icpengine.cpp:345-346; CLI :598-603)
 *   icp_hip_get_source   write-back of the source (icpengine.cpp:371-375; CLI :609-613)
 *   icp_hip_get_correspondences  `correspondences` vector (icpengine.cpp:169-179)
 *
 * Errors: every call returns ICP_HIP_OK (0) or a negative ICP_HIP_E* code; the message is in
 * icp_hip_last_error() (thread-local). Host buffers are borrowed for the duration of a call.
 * A context is driven by one host thread at a time.
 */
#ifndef ICP_HIP_H
#define ICP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICP_HIP_OK 0
#define ICP_HIP_EINVAL (-1)
#define ICP_HIP_ENOMEM (-2)
#define ICP_HIP_EDEVICE (-3)
#define ICP_HIP_ERCCL (-4)
#define ICP_HIP_ENOTREADY (-5)
#define ICP_HIP_EEXCHANGE (-6) /* the host-exchange callback (icp_hip_comm_init_host) failed or
                                  overran config.peer_timeout_ms */

#define ICP_HIP_UNIQUE_ID_BYTES 128

/* Which reference flavour an iteration follows (they differ in the octree's initial best
 * distance and the first-iteration threshold). */
#define ICP_RULES_ENGINE 0 /* core/icpengine.cpp: best = DBL_MAX, iter-0 relaxed threshold */
#define ICP_RULES_CLI 1    /* icp_registration.cpp: best = 1e20, threshold mean + 3 std  */

/* Search kernels. Both return the reference's correspondences bit for bit. */
#define ICP_SEARCH_CERTIFIED 0 /* wave-cooperative search + certificate (the product path)     */
#define ICP_SEARCH_REFERENCE 1 /* one thread per query, the literal reference-order DFS         */

#define ICP_BUILD_AUTO 0 /* octree built on the device (max_depth <= 21), else on the host       */
#define ICP_BUILD_HOST 1 /* always the host builder (same arrays bit for bit)                   */

/* Explicit configuration of a context (nothing is read from the environment). Every setting
 * gives the same correspondences; they select how the device finds them. */
typedef struct icp_hip_config {
  uint32_t config_version; /* ICP_HIP_CONFIG_VERSION, set by icp_hip_config_default. The FIRST word,
                              so create_ex checks it before it copies the struct: a struct of
                              another header version (v1/v2 began with `search`, 0 or 1) is
                              rejected without reading past the caller's object               */
  int32_t search;         /* ICP_SEARCH_*                                        default CERTIFIED */
  int32_t scan32;         /* 1: fp32 filter scan + fp64 certificate; 0: fp64 scan      default 1 */
  int32_t cell_starts;    /* 1: wave walks start from per-level cell tables; 0: root    default 1 */
  int32_t octree_builder; /* ICP_BUILD_*                                             default AUTO */
  double join_factor;     /* a query joins its wave's search box if its search radius is at most
                             join_factor x the wave's mean radius                      default 3.0 */
  int32_t debug_counters; /* 1: the wave search counts its phases (icp_hip_debug_counters) dflt 0 */
  int32_t xcd_blocks;     /* > 0: the wave search's blocks are renumbered so that each XCD (own
                             L2) takes runs of this many consecutive (spatially adjacent)
                             blocks, dealt round-robin over the XCDs; 0: hardware order  dflt 256 */
  int32_t scan_groups;    /* 1, 2 or 4: the fp32 filter scan of a wave splits its lanes into this
                             many kd sub-buckets, each scanning only the candidates inside its
                             own box; a wave that reuses its cache record stages its groups'
                             candidates across its chunks and scans once (fewer evaluations per
                             query against more staging work: at 4, 29 point pairs per wave
                             instead of 48 at 2; search 4-7 % faster on config 4)     dflt 4 */
  int32_t candidate_cache;  /* 1: each wave of the iterate's search keeps the candidate list of
                               its search box B enlarged by candidate_margin (1/256 units of B's
                               largest half-extent per side), and the next iterate reuses it
                               without walking the octree while its new box lies inside
                               (an exact containment test: results are unchanged); 0: every
                               iterate walks                                              dflt 1 */
  int32_t candidate_margin; /* see candidate_cache, in [0, 1024]                        dflt 16 */
  int32_t certify_prev;   /* after an iterate on the same queries, a query whose previous match p*
                             is certified by p*'s separation (a lower bound of p*'s distance to
                             every other target point, computed once per target) keeps it without
                             a search (exact: the window certificate of DESIGN.md §3.1).
                             0: off; 1: only waves whose every query is certified skip the search;
                             2: certified queries settle, the rest of the wave searches;
                             3: certified queries settle; a wave left with at most 4 open
                                queries hands them to the ball search, else searches them (2).
                             Pays off near convergence (residuals well below the point spacing);
                             on config 4's sliding synthetic pair ~0.2 % of the queries certify
                             and 1/2 cost +4 % search time          dflt 0 */
  int32_t query_order;    /* the kd order of the source queries (64-query buckets = waves):
                             0: built on the device; 1: on the host (query_order.cpp)  dflt 0 */
  int32_t overflow_halves; /* 1: in the first iterate of a source (descent guesses, ~16 % of
                              the waves overflow), the queries of a wave whose search box
                              overflows are searched again as two 32-query halves (k_nn_half)
                              before the wide pass / ball search; 0: the wide pass takes the
                              whole wave (wide_pass; measured better on the blob and the
                              scene: first iterate 2.45 -> 2.38 ms, 41 -> 29.6 ms)   dflt 0 */
  int32_t device_loop;    /* 1: the engine session's batches (icp_session_step_n, icp_engine_run)
                             run as a device-resident loop: each iteration's last kernel takes
                             the session's decisions and computes the transform (the host
                             loop's own code, session_step.h), so the iterations of a batch
                             run back to back with one host wait per batch (single-device
                             contexts; multi-device groups and the host exchange step on the
                             host); 0: the host steps every iteration. The device step (one
                             lane's fp64 Jacobi SVD, ~8.5 us) costs what the host round trip
                             does (7-11 us): equal at 10M and 1.25M shards, 5 % slower at 100k
                                                                            dflt 0 */
  int32_t timing_stride;  /* iterates whose search kernel is timed by events on its dispatch and the
                             next kernel's (icp_hip_timings): every timing_stride-th iterate of the
                             context (the first included); 0: none. An event on a dispatch packet
                             delays the next kernel by ~3-5 us (every iterate timed: config 2,
                             100k, 12-15 % slower)                                      dflt 0 */
  int32_t candidate_loose; /* a cached candidate list is reused only while vol(B+) <= this / 100 x
                              vol(B) (a wave whose box shrank walks again and stores a tighter
                              list; the same results either way), in [100, 100000]; 0: the
                              default. 1500 since r23: surface data's residuals shrink for
                              tens of iterates, and at 190 ~80 % of the scene's waves walked
                              again every iterate (search 1.03 -> 0.76 ms at 10M)  dflt 1500 */
  int32_t candidate_lead;  /* a walking wave of an iterate extends the B+ it stores, on each axis,
                              by this many times the displacement of B's centre by the
                              iterate's transform, on the side the queries moved to (ICP moves a
                              wave's queries the same way for many iterates: a record then lasts
                              until they have moved that far), in [0, 64]; 0: symmetric margin
                              only                                                       dflt 8 */
  int32_t fused_cull;      /* 1: from a source's second iterate on, the wave search also sums the
                              covariance terms of its pairs below a band around the previous
                              iterate's threshold, and the cull pass only settles the band and the
                              waves the search left to its other paths (icp_hip_last_cull_path);
                              0: every cull is a full pass. The same valid pairs either way; the
                              sums differ in their order only                             dflt 1 */
  int32_t peer_timeout_ms; /* multi-rank iterates (comm_init / comm_init_host): the longest the host
                              waits for an iterate whose record exchange involves peers. Past it
                              the iterate fails (RCCL: ICP_HIP_ERCCL after ncclCommAbort, so the
                              pending collective returns and the stream drains; host exchange:
                              ICP_HIP_EEXCHANGE, the callback left running on the context's
                              exchange thread) and every later iterate fails with ICP_HIP_ERCCL
                              until comm_init / comm_init_host. 0: no deadline. Independently of
                              it, an RCCL communicator's asynchronous error (a peer process that
                              died, a broken link: ncclCommGetAsyncError) is checked while the
                              host waits, with the same outcome                           dflt 0 */
  int32_t no_warmup;       /* 0: the first context a process creates on a device with a given set of
                              search options runs a 3-iterate registration of a 4096-point
                              synthetic pair on a private context first (~5 ms, once): HIP
                              loads a kernel's code and sizes its scratch at the kernel's first
                              launch, which otherwise lands in the first real iterate (+1.3 ms
                              at 10M); 1: no warm-up                                     dflt 0 */
  int32_t ball_mode;       /* k_nn_ball, the queries the wave search left: 0 a whole query per wave
                              (the cooperative search from the cell tables of its bound) when the
                              list is short (<= one per wave of the launch) or long (> four per
                              wave: an unconverged registration on surface data), else four
                              queries per wave (16-lane ball walks, follow-ups for the balls that
                              overflow); 1 always the ball walk; 2 always whole queries. The same
                              results either way                          dflt 0 */
  int32_t wide_pass;       /* the wave search's boxes that hold more candidates than its LDS list
                              (a box 10-100x denser than its queries: surface data far from
                              convergence, occlusion shadows): 0 (auto) searched again by the wide
                              pass (k_nn_wide: the same box walked and scanned in segments by the
                              same 64 lanes) in a source's first iterate and whenever the previous
                              iterate had >= max(256, waves / 32) such waves, else their queries
                              take the ball search; 1 never; 2 always. The same results either
                              way                                                          dflt 0 */
  int32_t reserved[3];     /* zero (fields of later versions of this header); create_ex rejects
                              a nonzero word                                                    */
} icp_hip_config;
#define ICP_HIP_CONFIG_VERSION 3u /* 1: r4 and earlier (no version field); 2: r5 (version last) */

/* Slots of icp_hip_debug_counters (summed over the last iterate's search launches). */
#define ICP_DBG_WAVES 0          /* waves of the wave search                                  */
#define ICP_DBG_OVERFLOW 1       /* waves whose candidate set overflowed LDS                   */
#define ICP_DBG_NOT_JOINED 2     /* lanes with a guess that did not join their wave's box      */
#define ICP_DBG_NOT_COVERED 3    /* joined lanes whose nearest point was beyond their guess    */
#define ICP_DBG_RESCAN_POINTS 4  /* points scanned by fp64 re-scans                            */
#define ICP_DBG_WALK_BATCHES 5   /* walk batches (up to 64 nodes each)                          */
#define ICP_DBG_NO_GUESS 6       /* lanes without a usable guess                               */
#define ICP_DBG_CANDIDATES 7     /* candidate points collected by the walks                    */
#define ICP_DBG_FP64_WAVES 8     /* waves re-scanned in fp64 (uncertified after the fp32 scan) */
#define ICP_DBG_STAGED 9         /* points staged for the fp32 scan                            */
#define ICP_DBG_SCAN_PAIRS 10    /* point pairs evaluated by the fp32 scan (per wave)          */
#define ICP_DBG_SCAN_ROUNDS 11   /* fp32 scan rounds                                           */
#define ICP_DBG_CACHE_HITS 12    /* waves that reused their cached candidate list              */
#define ICP_DBG_CACHE_STORES 13  /* waves that walked and stored their candidate list          */
#define ICP_DBG_BALL_OVERFLOW 14 /* ball-search queries whose candidate set overflowed         */
#define ICP_DBG_BALL_POINTS 15   /* points scanned by the ball search                          */
#define ICP_DBG_HALVES 16        /* 32-query halves of overflowed waves searched again (k_nn_half) */
#define ICP_DBG_CLK_GUESS 16     /* phase-clock build (-DICP_PHASE_CLOCKS=1), s_memtime: guess  */
#define ICP_DBG_REUSED_ENTRIES 17 /* cache entries streamed by the waves that reused their record */
#define ICP_DBG_CLK_BOX 17       /*                          search box                        */
#define ICP_DBG_CLK_WALK 18      /*                          walk (cells + batches)            */
#define ICP_DBG_CLK_SCAN 19      /*                          scan                              */
#define ICP_DBG_PREV_WAVES 18    /* count build: waves whose every query the previous-match
                                    certificate settled (certify_prev)                           */
#define ICP_DBG_PREV_LANES 19    /* count build: queries settled by the previous-match certificate */
#define ICP_DBG_CLK_FINISH 20    /*                          certify + write + queue           */
#define ICP_DBG_WINNER_PREV_WAVES 20 /* winner-count build (-DICP_WINNER_COUNTS=1): waves whose
                                        every fp32 winner is the lane's previous match          */
#define ICP_DBG_START_NODES 21   /* start nodes taken from the cell tables / descent levels    */
#define ICP_DBG_WINNER_PREV 22   /* winner-count build: joined lanes whose winner is the previous match */
#define ICP_DBG_WINNER_LANES 23  /* winner-count build: joined lanes with an fp32 winner          */
#define ICP_DBG_WALK_MOVED 24   /* waves with a record of this generation that walked because
                                    their box left B+                                        */
#define ICP_DBG_WALK_LOOSE 25   /* waves whose box lay inside B+ but walked because B+ was loose */
#define ICP_DBG_GROUP_POINTS 26 /* fp32 scan: points staged, summed over the scan groups       */
#define ICP_DBG_BB_QUERIES 27   /* ball-search follow-ups taken by the wave-cooperative search  */
#define ICP_DBG_BB_STEPS 28     /* their steps (up to 64 nodes each)                            */
#define ICP_DBG_LANE_HANDED 29  /* per-lane follow-ups that ran out of their node budget        */
#define ICP_DBG_FZ_RECOMPUTE 30 /* waves whose covariance record the cull recomputes (queries
                                   left to the other searches)                                 */
#define ICP_DBG_FZ_BAND 31      /* queries in the band around the previous threshold           */
#define ICP_DBG_WIDE_WAVES 32    /* waves (or halves) the wide pass searched again               */
#define ICP_DBG_WIDE_SEGMENTS 33 /* candidate-list segments the wide pass scanned                 */
#define ICP_DBG_WIDE_STACK 34    /* wide walks whose node stack overflowed (lanes to the ball search) */
#define ICP_DBG_WIDE_UNDECIDED 35 /* lanes the wide pass left to the ball search (no certificate) */
#define ICP_DBG_WIDE_POINTS 36   /* candidate points listed by the wide walks                      */
#define ICP_DBG_BB_OVERFLOW 37   /* cooperative searches whose frontier still outgrew the stack  */
#define ICP_DBG_LANE_EXACT 38    /* queries the ball search finished by the reference-order DFS
                                    after the cooperative search (a tie or an overflow)          */
#define ICP_DBG_SLOTS 40

typedef struct icp_hip_ctx icp_hip_ctx;

/* Statistics of one iteration, global over all ranks (identical on every rank). */
typedef struct icp_iter_stats {
  int64_t n;          /* source points (all ranks)                              */
  double mean;        /* mean residual                       icpengine.cpp:235-239 */
  double std;         /* population std of the residuals     icpengine.cpp:241-245 */
  double threshold;   /* cull threshold                      icpengine.cpp:249-255 */
  int64_t valid;      /* pairs with d <= threshold           icpengine.cpp:263-271 */
  double rmse;        /* sqrt(sum_valid d^2 / valid)         icpengine.cpp:274-278 */
  double sum_d2;
  double min_d, max_d;/* over finite residuals               icpengine.cpp:220-223 */
  int64_t n_bad;      /* non-finite residuals                icpengine.cpp:208-218 */
  double centroid_src[3]; /* mean of valid source points     icpengine.cpp:82     */
  double centroid_tgt[3]; /* mean of matched target points   icpengine.cpp:83     */
  double H[9];        /* sum (a-ca)(b-cb)^T row-major        icpengine.cpp:86-90  */
  int64_t n_fallback; /* this rank's queries the certified fast search handed to the exact
                         reference-order DFS (near-ties)                     */
  int64_t n_lane_search; /* this rank's queries left to the per-lane certified search (no
                            usable distance guess, or an overflowing one-query ball search)  */
  int64_t n_ball_search; /* this rank's queries a wave did not take (outliers, overflowing
                            waves), searched one query per wave around their guess            */
} icp_iter_stats;

int icp_hip_device_count(int* count);

void icp_hip_config_default(icp_hip_config* cfg);

/* Create a context on `device` (HIP ordinal; -1 = the calling thread's current device) with the
 * default configuration, or with `cfg` (null = default). */
int icp_hip_create(icp_hip_ctx** out, int device);
int icp_hip_create_ex(icp_hip_ctx** out, int device, const icp_hip_config* cfg);
void icp_hip_destroy(icp_hip_ctx* ctx);

/* Transports of a multi-device context (icp_hip_create_multi); icp_hip_ctx_devices also reports
 * ICP_XPORT_CALLBACK (icp_hip_comm_init_host) and ICP_XPORT_AUTO (= none: a world of one). */
#define ICP_XPORT_AUTO 0     /* RCCL when the device ids are distinct, else the host gather       */
#define ICP_XPORT_RCCL 1     /* communicators from ncclCommInitAll (distinct devices)            */
#define ICP_XPORT_HOST 2     /* in-process host gather (any ids: rehearses N ranks on one GPU)   */
#define ICP_XPORT_CALLBACK 3 /* the caller's exchange callback (icp_hip_comm_init_host)          */

/* One context driving n_devices GPUs from this process: the multi-GPU path behind the
 * single-process drop-in (ICPEngine::registerPointClouds, icpengine.cpp:24-60; CLI ICP(),
 * icp_registration.cpp:443-446; SURVEY.md §8b icp_hip_create(ctx, n_devices, device_ids)).
 * The source is sharded over the devices in spatially compact ranges (icp_source_shard_order),
 * the octree replicated; each device has a driver thread of its own, and the two per-iteration
 * exchanges are RCCL all-gathers over communicators from ncclCommInitAll (ICP_XPORT_RCCL) or an
 * in-process host gather (ICP_XPORT_HOST). Every other entry point of this header accepts the
 * returned context as it accepts a single-device one: outputs in the caller's order, statistics
 * identical on all devices (those of a world of n_devices processes), timings the slowest
 * device's, search-path counts summed. comm_init / comm_init_host do not apply to it. A source
 * needs at least one point per device (and fewer than 2^31 points in all). n_devices = 1 with
 * ICP_XPORT_AUTO gives a plain context.
 * Failures: a call that fails on one member returns that member's error (a peer's own
 * ICP_HIP_EEXCHANGE is not reported over the root cause); the next call starts clean. Except:
 * when an iterate fails over ICP_XPORT_RCCL, a peer may already have enqueued a collective that
 * will never complete, so every member's communicator is aborted (ncclCommAbort: the pending
 * collectives return) and the context is DEAD: every later call but icp_hip_destroy returns
 * ICP_HIP_EDEVICE. Destroy it and create a new one. (Usage errors found before any member runs,
 * e.g. no target or source, do not kill it.) */
int icp_hip_create_multi(icp_hip_ctx** out, int n_devices, const int* device_ids, const icp_hip_config* cfg,
                         int transport);
/* Devices (up to cap ids) and transport (ICP_XPORT_*) of a context. */
int icp_hip_ctx_devices(icp_hip_ctx* ctx, int32_t* n_devices, int32_t* device_ids, int32_t cap, int32_t* transport);

/* Multi-GPU: rank 0 calls get_unique_id, the caller distributes the bytes (any side channel),
 * then every rank calls comm_init. Without it a context is a world of one. A communicator of
 * one rank (nranks = 1) is created as well: every iteration then runs the multi-rank path
 * (RCCL all-gathers + rank-order merges) on a world of one. */
int icp_hip_get_unique_id(uint8_t out[ICP_HIP_UNIQUE_ID_BYTES]);
int icp_hip_comm_init(icp_hip_ctx* ctx, int nranks, int rank, const uint8_t id[ICP_HIP_UNIQUE_ID_BYTES]);

/* Multi-rank without RCCL: the two per-iteration all-gathers go through the caller's callback.
 * `exchange` receives this rank's record (`count` doubles) and fills `gathered` with every
 * rank's record in rank order (nranks x count); it returns 0 on success. The rest of the
 * multi-rank path (rank-order merge on the device, publish) is the one comm_init runs. Used to
 * rehearse several ranks on one GPU (RCCL refuses two ranks on one device) and by callers that
 * already own a host transport. Slower than RCCL: the stream is synchronised around each call.
 * A failing callback makes icp_hip_iterate return ICP_HIP_EEXCHANGE; the peer ranks are then
 * left waiting inside their own exchange, and the caller must tear them down.
 * When icp_hip_iterate fails with ICP_HIP_EEXCHANGE or ICP_HIP_ERCCL, its T_apply has ALREADY
 * been applied to the resident source (the search kernel moves the queries before the exchange):
 * a caller that retries the iterate must pass T_apply = null. */
typedef int (*icp_hip_exchange_fn)(void* user, const double* local, int32_t count, double* gathered);
int icp_hip_comm_init_host(icp_hip_ctx* ctx, int nranks, int rank, icp_hip_exchange_fn exchange, void* user);

/* Abort this rank's RCCL communicator (ncclCommAbort): collectives it has enqueued that a failed
 * peer will never join return, so the stream drains and icp_hip_destroy cannot block. For a
 * rank whose peer failed (one process per GPU; the multi-device context does this itself). The
 * context's iterates (icp_hip_iterate and the device-resident loop of icp_session_step_n /
 * icp_engine_run) then fail with ICP_HIP_ERCCL until comm_init / comm_init_host is called
 * again. No communicator: nothing to do.
 * Peer failure without a call to this function: while the host waits for a multi-rank iterate
 * it checks the communicator's asynchronous error and config.peer_timeout_ms, and on either
 * aborts the communicator itself (the iterate returns ICP_HIP_ERCCL). A host-exchange callback
 * that overruns config.peer_timeout_ms makes the iterate return ICP_HIP_EEXCHANGE; the callback
 * keeps running on the context's exchange thread and must return eventually: comm_init,
 * comm_init_host and icp_hip_destroy wait for it. */
int icp_hip_comm_abort(icp_hip_ctx* ctx);

/* The communicator as RCCL itself reports it (ncclCommCount, ncclCommUserRank, ncclCommCuDevice)
 * for member `member` of a context (0 for a single-device context; a device group's members in
 * device-list order), and its transport (ICP_XPORT_RCCL, ICP_XPORT_CALLBACK for the host
 * exchange, ICP_XPORT_AUTO for none). Without an RCCL communicator: the context's own world size,
 * rank and device. Lets a launcher check that RCCL saw the world it asked for. Any output may be
 * null. Replaces nothing in the reference (single-process CPU code). */
int icp_hip_comm_info(icp_hip_ctx* ctx, int member, int32_t* count, int32_t* rank, int32_t* device,
                      int32_t* transport);

/* Time (ms) of the two per-iteration record all-gathers of each of the last k iterates (k <= 256),
 * oldest first: HIP events around the RCCL all-gathers on the compute stream (so the figure
 * includes waiting for the slowest peer to arrive), or the host clock around the host exchange's
 * callback. NaN for an iterate that config.timing_stride left untimed or that ran without peers.
 * A device group reports its slowest member per iterate. Waits for the iterates to finish. */
int icp_hip_exchange_timings(icp_hip_ctx* ctx, int k, double* exchange_ms);

/* Build the reference octree of the target (AoS xyz, n points) and keep it in HBM. The tree is
 * built on the device (max_depth <= 21, config octree_builder AUTO) or on the host (deeper
 * trees, or ICP_BUILD_HOST); both produce the same arrays bit for bit. rules selects the initial
 * best distance of findNearest. Non-finite target coordinates and empty targets are rejected
 * (ICP_HIP_EINVAL). Replaces Octree::Octree(points, max_pts, max_d), octree.cpp:41-126. */
int icp_hip_set_target(icp_hip_ctx* ctx, const double* xyz, int64_t n, int max_points, int max_depth,
                       int rules);

/* Which builder made the resident octree (1 = device) and the set_target time in ms. */
int icp_hip_target_build_info(icp_hip_ctx* ctx, int32_t* on_device, double* build_ms);

/* Copy the resident octree back in the layout of icp_octree_copy_nodes / _copy_points
 * (icp_host.h); sizes from icp_hip_target_info (nodes) and the target size (points). */
int icp_hip_copy_target(icp_hip_ctx* ctx, double* box6, int32_t* first, uint32_t* meta, int32_t* depth,
                        double* xyz, int32_t* orig);

/* The separation of every target point (caller's target order): a lower bound of its distance
 * to every other target point, 0 when it has an exact duplicate (computed by set_target when
 * config certify_prev != 0; zeros otherwise). Inspection / tests. */
int icp_hip_target_separation(icp_hip_ctx* ctx, float* sep_out);

/* Upload this rank's source shard (AoS xyz). Queries are reordered on the device along a
 * Morton curve for traversal coherence; every output is returned in the caller's order.
 * A shard holds fewer than 2^29 points (ICP_HIP_EINVAL otherwise; shard larger clouds over a
 * device group). */
int icp_hip_set_source(icp_hip_ctx* ctx, const double* xyz, int64_t n);

/* One ICP iteration body. If T_apply (row-major 4x4) is non-null, src = T_apply * src is applied
 * first (fused into the search kernel). `iter` and `rules` select the threshold rule,
 * sigma_multiplier is k in mean + k*std. Fills *out (identical on all ranks). */
int icp_hip_iterate(icp_hip_ctx* ctx, const double* T_apply, int iter, int rules, double sigma_multiplier,
                    icp_iter_stats* out);

/* src = T * src on the resident source (row-major 4x4). */
int icp_hip_apply(icp_hip_ctx* ctx, const double* T);

/* Copy the resident (transformed) source back, AoS, caller's order. */
int icp_hip_get_source(icp_hip_ctx* ctx, double* xyz_out);

/* Correspondences (original target indices) and residuals of the last iterate, caller's order.
 * Either pointer may be null. */
int icp_hip_get_correspondences(icp_hip_ctx* ctx, int32_t* idx_out, double* dist_out);

/* Parity hook: nearest target index + residual for arbitrary queries (AoS), no reordering,
 * no transform — exactly Octree::findNearest + computeDistance per query. */
int icp_hip_nn(icp_hip_ctx* ctx, const double* q_xyz, int64_t n, int32_t* idx_out, double* dist_out);

/* Work of the reference DFS for the resident source (node entries and leaf points compared,
 * both as the reference visits them) — the V and P of the roofline byte model. */
int icp_hip_traversal_counts(icp_hip_ctx* ctx, double* mean_node_entries, double* mean_leaf_points);

/* Shape of the uploaded octree. */
int icp_hip_target_info(icp_hip_ctx* ctx, int64_t* n_nodes, int64_t* n_leaves, int32_t* max_depth,
                        int32_t* stack_levels);

/* Time (ms, HIP events on the context's stream) of the last search-kernel launch, and of the
 * whole device part of the last iterate. ICP_HIP_ENOTREADY when config.timing_stride left the
 * last iterate untimed (the default timing_stride 0 times none: an event on a dispatch delays
 * the next kernel). */
int icp_hip_last_timing(icp_hip_ctx* ctx, double* nn_kernel_ms, double* iterate_device_ms);

/* The same for each of the last k iterates (k <= 256, the context's timing ring), oldest first;
 * NaN for an iterate that config.timing_stride left untimed.
 * Waits for them to finish. */
int icp_hip_timings(icp_hip_ctx* ctx, int k, double* nn_kernel_ms, double* iterate_device_ms);

/* Which pass produced the last host-published iterate's covariance sums: 1 = the wave search
 * summed its pairs below a band around the previous threshold and the cull pass only settled the
 * band and the waves the search left unfinished; 0 = a full cull pass (a source's first iterate,
 * a threshold outside the band, the reference-order search). The statistics are the same either
 * way up to the summation order. A multi-device context reports 1 when every member did.
 * ICP_HIP_ENOTREADY before the first iterate of a source. */
int icp_hip_last_cull_path(icp_hip_ctx* ctx, int32_t* fused);

/* The wave search's diagnostic counters of the last iterate (ICP_DBG_* slots); zeros unless the
 * context was created with debug_counters = 1. */
int icp_hip_debug_counters(icp_hip_ctx* ctx, uint64_t out[ICP_DBG_SLOTS]);

int icp_hip_synchronize(icp_hip_ctx* ctx);

/* Testing hook (failure paths of the multi-rank and multi-device iterate): the next iterate of
 * member `member` of a multi-device context (0 for a single-device one) fails with
 * ICP_HIP_EDEVICE just before its first record exchange, i.e. after its search and before it
 * joins the collective its peers are waiting in. where = 0 clears it. */
int icp_hip_debug_inject_failure(icp_hip_ctx* ctx, int member, int where);

const char* icp_hip_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
