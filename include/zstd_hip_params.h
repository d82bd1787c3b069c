/*
 * zstd_hip_params.h — constants that define the compressed bit stream of the
 * gfx950 path.  Shared by the HIP kernels (custom-nvcomp-with-zstd_amd/csrc)
 * and the CPU restatement used as the test oracle (oracle/zstd_oracle.c), so
 * that both run the same algorithm.  Changing any value changes the output
 * bytes (but never their decodability).
 *
 * Level-3 parameters follow the reference's level table
 * (src/cuda_zstd_types.cpp:158-164: DFAST, min_match 3, search depth 2) mapped
 * onto a deterministic, LDS-resident double-hash match finder.
 */
#ifndef ZSTD_HIP_PARAMS_H_
#define ZSTD_HIP_PARAMS_H_

#define ZH_BLOCK_MAX 65536          /* bytes per device block (one workgroup) */
#define ZH_HIST_BLOCK 32768         /* device block of a history frame (below) */
#define ZH_HIST_WINDOW_LOG 16       /* history needs a window of >= 64 KiB */
/* Device block size of a frame of n bytes: frames up to 64 KiB are one
 * block; larger frames are cut into 32 KiB blocks that are each staged behind the 32 KiB before
 * them (the previous block), so matches reach across block boundaries within the 64 KiB of LDS.
 * split_dict = a dictionary (or stream history) frame below ZH_DEEP_LEVEL: its first block is
 * staged behind the last 64 KiB - block bytes of the dictionary content, so frames over 32 KiB
 * are cut into 32 KiB blocks too (the first sees 32 KiB of dictionary, not 64 KiB - n).  The
 * deep matcher (levels >= ZH_DEEP_LEVEL) stages its prefix outside LDS and never splits.
 * Workspace sizes are taken for the split layout (a dictionary is not known when the temp size
 * is asked for; the reference's temp size does not depend on it either,
 * src/cuda_zstd_manager.cu:5661). */
#define ZH_FRAME_BLOCK(n, split_dict) ((n) <= ((split_dict) ? ZH_HIST_BLOCK : ZH_BLOCK_MAX) ? ZH_BLOCK_MAX : ZH_HIST_BLOCK)
#define ZH_TILE 128                 /* hash insertion granularity (positions) */
#define ZH_WINDOW 2048              /* parse window (positions); catch-up stays inside one */
#define ZH_SKIP_TILES 2             /* tiles a window searches after a window without matches (miss skip);
                                       a match among them resumes the search of the whole window */
#ifndef ZH_PROBE_WINDOWS
#define ZH_PROBE_WINDOWS 1          /* a block whose parse takes no match in its first windows is all literals */
#endif
/* The probe applies only when its window holds at least ZH_WINDOW - ZH_PROBE_MAX_E0 block
 * positions (a block whose `pre` sits late in its window is never probed). */
#define ZH_PROBE_MAX_E0 (ZH_WINDOW / 2)
/* Repeat scan: a block the probe finds no match in is all literals only when this whole-block
 * test also finds (almost) no repeated 8-byte string.  Positions q = 0 mod ZH_SCAN_STRIDE of the
 * staged buffer (history included) are entered into a 2^ZH_SCAN_LOG-slot table keyed by the long
 * hash's top bits, each slot keeping the minimum of (16 more bits of the hash) << 16 | q; the block
 * positions p = pre + ZH_SCAN_STEP m are looked up, and p counts when its slot's entry carries p's
 * 16 bits and a position below p.  With the strides coprime, every repeat of at least 8 +
 * ZH_SCAN_STRIDE x ZH_SCAN_STEP bytes has a sampled pair.  The block is resurrected (parsed in full,
 * no probe) when at least max(ZH_SCAN_MIN, block positions >> ZH_SCAN_SHIFT) positions count. */
#define ZH_SCAN_LOG 14
#define ZH_SCAN_STRIDE 4
#define ZH_SCAN_STEP 3
#define ZH_SCAN_SHIFT 12
#define ZH_SCAN_MIN 8
#define ZH_HASH_LOG_LONG 14         /* 8-byte hash table: 2^14 u16 entries */
#define ZH_HASH_LOG_SHORT 14        /* 5-byte hash table: 2^14 u16 entries */
#define ZH_HASH_READ 8              /* bytes read per hashed position */
/* K1's parse mode by level (levels 1-4; SURVEY.md §8f F2, reference level table
 * src/cuda_zstd_types.cpp:147-210): 0 = both tables + lazy-1 check (levels 3-4), 1 = the short
 * table only + lazy-1 (level 2), 2 = the short table only, greedy (level 1).  Oracle on the C3
 * mix (256 chunks; libzstd at that level): mode 2 2.647 (L1 2.534), mode 1 2.682 (L2 2.673),
 * mode 0 2.796 (L3 2.791). */
#define ZH_K1_MODE(level) ((level) <= 1 ? 2 : (level) == 2 ? 1 : 0)
/* Level 1's search stride (mode 2; libzstd fast's idea of not searching every
 * position): every position is still inserted into the short table, but only positions
 * p = 0 mod ZH_L1_STRIDE of the staged buffer look a match up -- a repeat is found at most
 * ZH_L1_STRIDE - 1 bytes late and the catch-up takes those bytes back -- so K1's length phase
 * runs NROUND / ZH_L1_STRIDE rounds per window.  Measured (C3 mix, 16,384 chunks, round 6,
 * profiles/r06b_level1_stride.json): stride 1 K1 9.51 ms, 84.0 GB/s, ratio 2.622; stride 2 8.05 ms,
 * 96.3 GB/s, 2.477 (libzstd L1 2.477); stride 4 7.42 ms, 102.7 GB/s, 2.271. */
#ifndef ZH_L1_STRIDE
#define ZH_L1_STRIDE 2
#endif
#define ZH_MIN_MATCH_LONG 8
#define ZH_MIN_MATCH_SHORT 5
#define ZH_MAX_MATCH 64             /* per-position length cap; continuations are merged */
/* Hashes: sums of 24 x 24-bit products (low 32 bits; gfx950 v_mad_u32_u24 runs at the full VALU
 * rate, a 64-bit multiply takes three quarter-rate v_mul_lo/hi_u32), top ZH_HASH_LOG bits.
 * Long (bytes 0..7): bytes 0-2, 3-5, 6-7 times ZH_HK_L0..2; short (bytes 0..4): bytes 0-2, 3-4
 * times ZH_HK_S0..1.  Same ratio as libzstd's 64-bit multiplicative hashes on the C3 mix
 * (tools/lz3_model.c: 2.7584 vs 2.7585). */
#define ZH_HK_L0 0x9E3779u
#define ZH_HK_L1 0x85EBCAu
#define ZH_HK_L2 0xC2B2AEu
#define ZH_HK_S0 0x27D4EBu
#define ZH_HK_S1 0x165667u
/* Deep matcher, levels >= ZH_DEEP_LEVEL (reference level table
 * src/cuda_zstd_types.cpp:172-183, matcher src/lz77_parallel.cu:26-70): exact hash chains over
 * the whole staged buffer (a dictionary frame's first block is staged behind the last
 * ZH_DEEP_PRE bytes of the dictionary content), keyed by the 5-byte short hash; per position the
 * longest of the first ZH_DEEP_DEPTH(level) chain candidates within ZH_DEEP_MAXOFF (>=
 * ZH_MIN_MATCH_SHORT bytes, capped at ZH_MAX_MATCH, nearest on ties); LAZY2 parse on those
 * matches, no catch-up. */
/* Levels 5-8 take the deep matcher at a smaller depth (the reference's level table gives them
 * 4-32 search steps, src/cuda_zstd_types.cpp:147-210): oracle on the C3 mix (256 chunks; libzstd
 * at that level in brackets): depth 4 2.810 (L5 2.817), 8 2.847 (L6 2.871), 16 2.881 (L7 2.890),
 * 32 2.910 (L8 2.923, L9 2.950).  Levels 1-4 run the dual-hash K1 (level 3's parse: 2.796, libzstd
 * L3/L4 2.791). */
#define ZH_DEEP_LEVEL 5
#define ZH_DEEP_PRE 65536
#define ZH_DEEP_MAXOFF 65535       /* links stored as u16 distances (zh_lz_deep.hip) are exact */
#define ZH_DEEP_DEPTH(level) ((level) <= 5 ? 4 : (level) == 6 ? 8 : (level) == 7 ? 16 : (level) <= 9 ? 32 : (level) == 10 ? 64 : 128)
#define ZH_COMPRESS_LITERALS_SIZE_MIN 63
#define ZH_LONGNBSEQ 0x7F00
#define ZH_MAGIC 0xFD2FB528u

#endif
