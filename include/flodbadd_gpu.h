/*
 * flodbadd_gpu.h -- C ABI of the MI355X (gfx950) packet-parse + flow-classification path.
 *
 * Drop-in boundary for edamametechnologies/flodbadd (reference @ 2025-07-18).  The reference
 * calls two Rust functions per captured frame from its capture task:
 *
 *   src/capture.rs:1038  parse_packet_pcap(&data)          -> Option<ParsedPacket>
 *   src/capture.rs:1046  process_parsed_packet(cp, &sessions, &current_sessions,
 *                                              &own_ips, &filter, l7)
 *   (async-capture twin at src/capture.rs:1224-1238)
 *
 * This header replaces that per-packet pair with batched, stream-ordered calls over a packed
 * frame buffer.  Every entry point is plain C (pointers + sizes, no torch/HIP types in the
 * signatures; streams are passed as `void*` = hipStream_t, NULL = the null stream).
 *
 * Conventions (mirroring the reference's error behaviour):
 *   - Every int-returning function returns FB_OK (0) or a negative fb_err; nothing aborts.
 *   - A frame the reference would reject (`parse_packet_pcap` returning None, src/packets.rs:
 *     603-802) is NOT an error: it is classified FB_CLASS_DROP.  A session packet rejected by
 *     the session filter (src/packets.rs:321-327) is FB_CLASS_FILTERED.  Port-53 traffic is
 *     FB_CLASS_DNS (src/packets.rs:638-650, 681-686) and is listed in the DNS side output.
 *   - A context is not thread-safe; use one per capture interface / stream, like the
 *     reference's one processor task per interface (src/capture.rs:1027).
 *   - Frames: `frames[offsets[i] .. offsets[i+1])` is frame i (caplen bytes, as libpcap hands
 *     `packet.data` to the reference, src/capture.rs:1092).  offsets has n+1 entries.
 *     A frame whose offsets are decreasing or exceed frames_bytes is classified DROP and
 *     counted in fb_batch_stats.bad_offsets.  Batches are limited to FB_MAX_BATCH_PACKETS
 *     packets and < 4 GiB of frame bytes (u32 offsets).
 */
#ifndef FLODBADD_GPU_H
#define FLODBADD_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FB_ABI_VERSION 4u /* 4: fb_flow_rec.segment_count / in_segment (136 B); 3: session_flags, error-word
                              bit 16, fb_flow_export_sessions* */
#define FB_MAX_BATCH_PACKETS ((1u << 27) - 1u)
#define FB_MAX_LAN_V6 64u  /* interface IPv6 (prefix, network) pairs, src/ip.rs:164-191 */
#define FB_MAX_OWN_IPS 64u /* per-interface own addresses, src/capture.rs:964-970      */
#define FB_SERVICE_BITMAP_BYTES 8192u
#define FB_MAX_FLOW_CAPACITY (1ull << 25) /* slots: 65,536 partitions of 512 (4 GiB of table)   */
#define FB_CFG_FIXED_TABLE 1u             /* fb_config.flags: never grow the flow table         */
#define FB_CFG_TIMED 2u                   /* fb_config.flags: capture-time state (fb_flow_time);
                                             every update call then needs fb_set_frame_times   */

/* Return codes. */
enum fb_err {
    FB_OK = 0,
    FB_ERR_INVAL = -1,      /* bad argument (NULL, size limits, bad enum)                 */
    FB_ERR_NOMEM = -2,      /* device or host allocation failed                           */
    FB_ERR_HIP = -3,        /* HIP runtime error; fb_last_error() has the text             */
    FB_ERR_NODEV = -4,      /* no gfx950 device / device index out of range                */
    FB_ERR_TABLE_FULL = -5, /* flow table capacity exhausted (some packets not counted)    */
    FB_ERR_INTERNAL = -6    /* kernel-side protocol failure (bounded spin expired)          */
};

/* SessionFilter, src/sessions.rs:173-178 (same discriminant order as the Rust enum). */
enum fb_filter { FB_FILTER_LOCAL_ONLY = 0, FB_FILTER_GLOBAL_ONLY = 1, FB_FILTER_ALL = 2 };

/* Per-packet class (the reference's Option<ParsedPacket> + filter outcome). */
enum fb_class {
    FB_CLASS_SESSION = 0,  /* ParsedPacket::SessionPacket that passed the filter -> out[]   */
    FB_CLASS_DNS = 1,      /* ParsedPacket::DnsPacket -> dns[]                              */
    FB_CLASS_DROP = 2,     /* parse_packet_pcap returned None                               */
    FB_CLASS_FILTERED = 3  /* SessionPacket rejected by the Local/Global filter             */
};

/* fb_pkt_out.meta bits. */
enum fb_meta_bits {
    FB_META_HAS_FLAGS = 1u << 0,  /* SessionPacketData.flags is Some (TCP)                  */
    FB_META_SWAP = 1u << 1,       /* canonical key = reversed raw 5-tuple                    */
    FB_META_ORIGINATOR = 1u << 2, /* is_originator, src/packets.rs:316-319                   */
    FB_META_LOCAL_SRC = 1u << 3,  /* is_lan_ip(key.src_ip), src/packets.rs:430               */
    FB_META_LOCAL_DST = 1u << 4,  /* is_lan_ip(key.dst_ip), src/packets.rs:431               */
    FB_META_SELF_SRC = 1u << 5,   /* own_ips.contains(key.src_ip), src/packets.rs:434        */
    FB_META_SELF_DST = 1u << 6,   /* own_ips.contains(key.dst_ip), src/packets.rs:435        */
    FB_META_DST_SERVICE = 1u << 7 /* dst_service is Some, src/packets.rs:441-464             */
};

/*
 * Session key, byte-identical to the reference's only C-ABI 5-tuple:
 * `struct session_key` (ebpf/l7_ebpf_program/src/l7_ebpf.c:26-34), mirrored by
 * `SessionKey` + `session_to_key` (src/l7_ebpf.rs:33-42, 78-104):
 *   IPv4: ip[0] = u32::from(Ipv4Addr) (numeric value, host byte order), ip[1..3] = 0.
 *   IPv6: ip[k] = u32::from_be_bytes(octets[4k..4k+4]).
 *   family from src_ip: 2 (AF_INET) / 10 (AF_INET6); protocol 6 (TCP) / 17 (UDP).
 */
typedef struct fb_session_key {
    uint32_t src_ip[4];
    uint32_t dst_ip[4];
    uint16_t src_port;
    uint16_t dst_port;
    uint8_t protocol;
    uint8_t family;
    uint16_t padding; /* always 0 */
} fb_session_key;     /* 40 bytes */

/*
 * One emitted session packet (class SESSION), in packet order.  Replaces the
 * SessionPacketData that reaches the DashMap upsert (src/packets.rs:85-98, 329-535).
 * `key` is the CANONICAL session key (src/packets.rs:245-311); the raw 5-tuple is `key`
 * reversed when FB_META_SWAP is set.
 */
typedef struct fb_pkt_out {
    fb_session_key key;        /*  0: canonical Session                                      */
    uint32_t packet_length;    /* 40: L4 payload bytes (SessionPacketData.packet_length)       */
    uint32_t ip_packet_length; /* 44: IPv4 total_length / IPv6 payload_length + 40             */
    uint8_t tcp_flags;         /* 48: TCP flags byte (0 when !HAS_FLAGS)                       */
    uint8_t meta;              /* 49: fb_meta_bits                                             */
    uint8_t hist_char;         /* 50: map_tcp_flags() char (src/packets.rs:561-601), 0 for UDP */
    uint8_t reserved;          /* 51: 0                                                        */
    uint32_t pkt_index;        /* 52: index of the frame in the batch                          */
} fb_pkt_out;                  /* 56 bytes */

/*
 * One SessionPacketData (src/packets.rs:92-98) -- the input of process_parsed_packet
 * (src/packets.rs:202) -- for hosts that keep their own decode and batch only the
 * classification + session-table part.  `session` is the Session AS PARSED (src = sender,
 * not canonicalised), in session_key layout; has_flags = flags.is_some().
 */
typedef struct fb_parsed_pkt {
    fb_session_key session;    /*  0 */
    uint32_t packet_length;    /* 40: L4 payload bytes                                        */
    uint32_t ip_packet_length; /* 44                                                          */
    uint8_t tcp_flags;         /* 48                                                          */
    uint8_t has_flags;         /* 49: 1 = Some(flags)                                          */
    uint16_t reserved;         /* 50: 0                                                        */
    uint32_t pkt_index;        /* 52: copied to fb_pkt_out.pkt_index                           */
} fb_parsed_pkt;               /* 56 bytes */

/* One DNS-diverted packet: payload = frames[payload_offset .. +payload_length). */
typedef struct fb_dns_out {
    uint32_t pkt_index;
    uint32_t payload_offset; /* absolute byte offset in the frame buffer; TCP: after the 2-byte
                                length prefix (src/packets.rs:646-647)                       */
    uint32_t payload_length;
    uint8_t protocol; /* 6 / 17 */
    uint8_t family;   /* 2 / 10 */
    uint16_t reserved;
} fb_dns_out; /* 16 bytes */

/* PACKET_STATS (src/packets.rs:28-83, 211-227, 336, 346) + batch bookkeeping. */
typedef struct fb_batch_stats {
    uint64_t total_processed; /* SessionPackets reaching process_parsed_packet (pre-filter)  */
    uint64_t tcp_processed;
    uint64_t udp_processed;
    uint64_t ipv4_processed;
    uint64_t ipv6_processed;
    uint64_t new_sessions;     /* flow-table inserts  (fb_flow_update only)                   */
    uint64_t updated_sessions; /* flow-table hits     (fb_flow_update only)                   */
    uint64_t n_session;        /* records written to out[] (class SESSION)                    */
    uint64_t n_dns;            /* records written to dns[] (class DNS)                        */
    uint64_t n_drop;           /* parse_packet_pcap -> None                                   */
    uint64_t n_filtered;       /* rejected by the session filter                              */
    uint64_t bad_offsets;      /* frames with invalid offsets (counted in n_drop too)         */
    uint64_t error;            /* nonzero = failure bits: 2 the two-pass dense path's offset scan
                                  waited too long (its records are not trusted and the update
                                  that follows skips them; FB_ERR_INTERNAL, not expected),
                                  4 flow-table partition full (FB_ERR_TABLE_FULL), 8 more records
                                  than the update scratch of the last parse launch holds,
                                  16 a table-update LDS spin expired (FB_ERR_INTERNAL),
                                  32 a dense tile offset put records past the batch (those
                                  records dropped, never written outside the buffers;
                                  FB_ERR_INTERNAL, not expected)                          */
    uint64_t reserved[3];
} fb_batch_stats; /* 128 bytes */

/* IPv6 LAN network (init_local_cache, src/ip.rs:164-191): ip & mask(prefix) == net. */
typedef struct fb_lan_v6 {
    uint32_t net[4]; /* network address, session_key word format (already masked)          */
    uint32_t prefix; /* 0..128                                                               */
    uint32_t reserved[3];
} fb_lan_v6; /* 32 bytes */

/* One own address (FlodbaddInterface v4/v6 addresses, src/capture.rs:964-970). */
typedef struct fb_ip {
    uint32_t addr[4]; /* session_key word format */
    uint32_t family;  /* 2 / 10 */
    uint32_t reserved[3];
} fb_ip; /* 32 bytes */

typedef struct fb_config {
    uint32_t abi_version;          /* must be FB_ABI_VERSION                                  */
    uint32_t filter;               /* fb_filter; FlodbaddCapture::new() uses GLOBAL_ONLY      */
    const uint8_t* service_bitmap; /* FB_SERVICE_BITMAP_BYTES; NULL -> built-in table
                                      (src/port_vulns_db.rs, bit p <=> name(p) != "")        */
    const fb_lan_v6* lan_v6;       /* may be NULL when n_lan_v6 == 0                          */
    uint32_t n_lan_v6;             /* <= FB_MAX_LAN_V6                                        */
    uint32_t n_own_ips;            /* <= FB_MAX_OWN_IPS                                       */
    const fb_ip* own_ips;          /* may be NULL when n_own_ips == 0                         */
    uint64_t flow_capacity;        /* INITIAL flow-table slots: rounded up to a power of two
                                      >= 512, at most FB_MAX_FLOW_CAPACITY; 0 = no table.
                                      Stored as partitions of 512 slots chosen by the key hash.
                                      The table grows (x2, rehashed on the device, before an
                                      update call) when the occupancy the last completed updates
                                      reported, projected over the updates still in flight,
                                      would fill a partition: the reference's map is unbounded
                                      (src/packets.rs:330).  A partition that still fills inside
                                      one batch reports error bit 4 (FB_ERR_TABLE_FULL)      */
    uint32_t max_batch_packets;    /* host-mode staging capacity (packets per call)           */
    uint32_t flags;                /* FB_CFG_*                                                */
    uint64_t max_batch_bytes;      /* host-mode staging capacity (frame bytes per call)       */
} fb_config;

/* determine_conn_state (src/packets.rs:539-559) outcome, fixed at the flow's first FIN/RST
 * packet (src/packets.rs:192-197, 422-426). */
enum fb_conn_state {
    FB_CONN_NONE = 0, /* conn_state None: no FIN/RST seen yet */
    FB_CONN_SF = 1,
    FB_CONN_S0 = 2,
    FB_CONN_REJ = 3,
    FB_CONN_S1 = 4,
    FB_CONN_OTHER = 5 /* "-" */
};

/* fb_flow_rec.hist_mask: bit k set <=> the history string contains FB_HIST_CHARS[k]
 * (map_tcp_flags alphabet, src/packets.rs:561-601). */
#define FB_HIST_CHARS "SsHhFfRr><Aa-"

/* A packet position in the stream of flow updates of one context: (update call << 32) | pkt_index,
 * where the update call counts fb_flow_update*_dev / fb_process*_dev calls since fb_create /
 * fb_flow_clear (from 0).  Stands for the wall-clock `now` the reference samples per packet
 * (src/packets.rs:209) -- a host maps it to capture timestamps.  FB_SEEN_NONE = None. */
#define FB_SEEN_NONE 0xFFFFFFFFFFFFFFFFull
#define FB_CALL_NONE 0xFFFFFFFFu /* fb_flow_mrec.char_call: the character has not occurred */

/* Flow-table export record: canonical key + SessionStats integer counters
 * (src/sessions.rs:76-82; update rules src/packets.rs:111-120, 383-391) + the ordered per-flow
 * state (src/packets.rs:187-198, 410-426): positions stand for start_time / last_activity /
 * end_time, hist_len = history.len(), conn_state as above.  The history string itself comes from
 * fb_flow_history_dev, batch by batch. */
typedef struct fb_flow_rec {
    fb_session_key key;      /*   0 */
    uint64_t outbound_bytes; /*  40 */
    uint64_t inbound_bytes;  /*  48 */
    uint64_t orig_pkts;      /*  56 */
    uint64_t resp_pkts;      /*  64 */
    uint64_t orig_ip_bytes;  /*  72 */
    uint64_t resp_ip_bytes;  /*  80 */
    uint64_t first_seen;     /*  88: position of the flow's first packet (start_time)         */
    uint64_t last_seen;      /*  96: position of its latest packet (last_activity)            */
    uint64_t end_seen;       /* 104: position of its first FIN/RST packet (end_time), or NONE */
    uint32_t hist_len;       /* 112: history.len() (TCP packets of the flow)                  */
    uint16_t hist_mask;      /* 116: characters present in history (FB_HIST_CHARS bits)       */
    uint8_t conn_state;      /* 118: fb_conn_state                                             */
    uint8_t end_mask;        /* 119: hist_mask & 0xFF at end_seen (the characters S s H h F f R r
                                conn_state was decided on); 0 while end_seen is NONE              */
    uint32_t slot;           /* 120: table slot (the flow id of fb_flow_history_dev)           */
    uint32_t session_flags;  /* 124: fb_session_flags as stored when the session was inserted
                                (src/packets.rs:429-435: is_local_src/dst, is_self_src/dst of the
                                canonical key under the configuration of that update call; and
                                dst_service is Some, src/packets.rs:441-466)                      */
    uint32_t segment_count;  /* 128: SessionStats.segment_count -- TCP packets with PSH: 1 for a
                                PSH first packet (src/packets.rs:414-420), +1 per later one
                                (140-160)                                                          */
    uint8_t in_segment;      /* 132: SessionStats.in_segment -- 0 right after a TCP PSH packet, 1
                                after any other (src/packets.rs:151-159, 376, 418)                 */
    uint8_t reserved[3];     /* 133 */
} fb_flow_rec;               /* 136 bytes.  Segment state under the no-timeout model: the
                                reference also ends a segment when a packet arrives >= 5 s of wall
                                clock after the flow's last one (segment_timeout, src/packets.rs:
                                137-149, 182-185); positions carry no clock.        */

/* Capture-time state of a flow on a timed context (fb_config.flags FB_CFG_TIMED; per-frame capture
 * timestamps handed to every update call with fb_set_frame_times).  The reference samples the wall
 * clock per packet (`now = Utc::now()`, src/packets.rs:230) and keeps, per session, start_time,
 * last_activity, end_time and the segment state (src/packets.rs:137-186 update, 352-380 + 414-426
 * insert): a TCP packet with PSH ends a segment, and so does any packet arriving >= 5 s
 * (segment_timeout, src/packets.rs:379) after the flow's previous one while a segment is open, which
 * then opens a new segment at that packet.  Here `now` is the frame's capture timestamp (ns), so the
 * state is a deterministic function of the input; chrono's num_milliseconds (truncation toward zero)
 * is applied to the same differences.  segment_count / in_segment of fb_flow_rec carry the timed state
 * on a timed context.  The reference accumulates total_segment_interarrival as an f64 running sum of
 * (ms / 1000.0) terms; this keeps the exact integer sum of the ms terms (the f64 running sum differs
 * from total_ms / 1000.0 by its own rounding, at most ~n ulp) and the divisor of the last accepted
 * term, so segment_interarrival = total_ms / 1000.0 / div (0.0 when div is 0). */
typedef struct fb_flow_time {
    uint64_t start_time_ns;            /*  0: SessionStats.start_time (the insert packet's time)      */
    uint64_t last_activity_ns;         /*  8: the flow's latest packet's time (arrival order)         */
    uint64_t end_time_ns;              /* 16: first FIN/RST packet's time; FB_SEEN_NONE = None          */
    uint64_t current_segment_start_ns; /* 24 */
    uint64_t last_segment_end_ns;      /* 32: FB_SEEN_NONE = None                                       */
    int64_t total_segment_interarrival_ms; /* 40: sum of the accepted segment interarrivals (ms)   */
    uint32_t segment_interarrival_div; /* 48: segment_count - 1 when the last term was accepted      */
    uint32_t segment_count;            /* 52: SessionStats.segment_count (timed)                       */
    uint8_t in_segment;                /* 56 */
    uint8_t reserved[3];               /* 57 */
    uint32_t slot;                     /* 60: table slot (joins fb_flow_rec.slot)                      */
} fb_flow_time;                        /* 64 bytes */
#define FB_SEGMENT_TIMEOUT_MS 5000 /* segment_timeout: 5.0 s, src/packets.rs:379 */

/* fb_flow_rec.session_flags (SessionInfo.is_local_src / is_local_dst / is_self_src / is_self_dst,
 * src/sessions.rs:40-61, set once at insert, src/packets.rs:429-435; bits 0-3 have the same values
 * as fb_enrich_bits) and FB_SESSION_DST_SERVICE: SessionInfo.dst_service is Some, i.e. the
 * service-port table names the canonical key's dst port at insert (src/packets.rs:441-466). */
enum fb_session_flags {
    FB_SESSION_LOCAL_SRC = 1u,
    FB_SESSION_LOCAL_DST = 2u,
    FB_SESSION_SELF_SRC = 4u,
    FB_SESSION_SELF_DST = 8u,
    FB_SESSION_DST_SERVICE = 16u
};

typedef struct fb_ctx fb_ctx;

/* ---- lifecycle ------------------------------------------------------------------------ */
uint32_t fb_abi_version(void);
const char* fb_last_error(void); /* thread-local text of the last failure */
fb_ctx* fb_create(int device, const fb_config* cfg); /* NULL on failure (see fb_last_error) */
int fb_destroy(fb_ctx* ctx);

/* ---- runtime configuration (each takes effect for the next call on the context) -------- */
int fb_set_filter(fb_ctx* ctx, uint32_t filter);                 /* set_filter, capture.rs:185 */
int fb_set_service_bitmap(fb_ctx* ctx, const uint8_t* bitmap);   /* CloudModel update, port_vulns.rs:350-380 */
int fb_set_lan_v6(fb_ctx* ctx, const fb_lan_v6* nets, uint32_t n); /* init_local_cache, ip.rs:164 */
int fb_set_own_ips(fb_ctx* ctx, const fb_ip* ips, uint32_t n);
/* Profiling hook (the reference's PACKET_STATS timing role, src/packets.rs:28-83): when `event`
 * (from fb_event_create, caller-owned; NULL clears) is set, fb_process_dev / fb_process_seg_dev
 * record it on their stream between the parse and the session-table update. */
int fb_set_stage_event(fb_ctx* ctx, void* event);
/* Timed contexts (FB_CFG_TIMED): the per-frame capture timestamps of the NEXT update call
 * (fb_flow_update*_dev, fb_process*_dev incl. the async and parsed-packet forms, fb_process_parsed):
 * d_ts[i] = frame i's capture time in ns since the Unix epoch (pcap header time, as the reference's
 * Utc::now() would read it), indexed by the records' pkt_index -- a DEVICE pointer that must stay
 * valid until that call's work completes on its stream (for fb_process_seg_async_dev: until
 * fb_flow_join or a later call's wait on it).  Consumed by that call; an update call on a timed
 * context without it fails with FB_ERR_INVAL before doing anything. */
int fb_set_frame_times(fb_ctx* ctx, const uint64_t* d_ts);
/* Test / diagnostic knobs of one context (never needed in production; each takes effect for the
 * next call): FB_DEBUG_DENSE_STEAL_POLLS -- the polls a dense look-back waits for a predecessor's
 * word before computing that tile's sums itself (default 4096; 0 forces the fallback path);
 * FB_DEBUG_DENSE_OFFSET_SKEW -- fault injection, added (mod 2^32) to the session half of every
 * dense tile offset, as a corrupted look-back word would be (< 2^32; logged on stderr when set). */
enum fb_debug_knob { FB_DEBUG_DENSE_STEAL_POLLS = 1, FB_DEBUG_DENSE_OFFSET_SKEW = 2 };
int fb_debug_set(fb_ctx* ctx, uint32_t knob, uint64_t value);
/* Whether the fused parse + upsert calls (fb_process_seg_dev, fb_process_seg_async_dev) store the
 * SESSION records in d_out (default 1).  With 0 the session table is their only per-packet output,
 * as in the reference's capture loop, which drops each ParsedPacket once process_parsed_packet has
 * updated the DashMap (src/capture.rs:1036-1061): d_out then receives only the DNS side records at
 * the segment tails, d_seg / d_class / d_stats are unchanged, and the history, export and
 * enrichment calls work as before (the update reads the parse's own update entries either way). */
int fb_set_session_records(fb_ctx* ctx, int emit);

/*
 * Device-resident parse + classify (parse_packet_pcap + the per-packet part of
 * process_parsed_packet).  All pointers are DEVICE pointers; the call is asynchronous on
 * `stream`.  Outputs, all optional except d_stats:
 *   d_out   : >= n fb_pkt_out, class-SESSION records, packet order (stable compaction)
 *   d_dns   : >= n fb_dns_out, class-DNS records, packet order
 *   d_class : n bytes, fb_class of every frame
 *   d_stats : one fb_batch_stats (overwritten, not accumulated)
 * One pass (k_parse_dense): 512-frame tiles whose batch-wide offsets come from a decoupled
 * look-back; a look-back that finds a predecessor tile unpublished for long computes that tile's
 * counts itself instead of waiting on it, so the call never depends on every workgroup being
 * resident and is safe on a GPU shared with other work.
 */
int fb_parse_classify_dev(fb_ctx* ctx, const uint8_t* d_frames, uint64_t frames_bytes,
                          const uint32_t* d_offsets, uint32_t n, fb_pkt_out* d_out,
                          fb_dns_out* d_dns, uint8_t* d_class, fb_batch_stats* d_stats,
                          void* stream);

/*
 * Host-memory variant: host buffers in, host buffers out (staged through the context's
 * pinned buffers with hipMemcpyAsync H2D/D2H).  Synchronous: returns after the results are
 * in host memory.  `out`/`dns` need room for n records; *n_out / *n_dns receive the counts.
 * Any of out, dns, cls, stats may be NULL.
 */
int fb_parse_classify(fb_ctx* ctx, const uint8_t* frames, uint64_t frames_bytes,
                      const uint32_t* offsets, uint32_t n, fb_pkt_out* out, uint32_t* n_out,
                      fb_dns_out* dns, uint32_t* n_dns, uint8_t* cls, fb_batch_stats* stats,
                      void* stream);

/*
 * Flow-table upsert of SESSION records (the DashMap entry()/update_session_stats part of
 * process_parsed_packet, src/packets.rs:329-535, integer counters only).  d_recs/d_n are
 * device pointers; the record count is read on the device from d_stats->n_session of the
 * fb_parse_classify_dev call that produced them, so no host round trip is needed.
 * new_sessions / updated_sessions are ADDED into d_stats.
 */
int fb_flow_update_dev(fb_ctx* ctx, const fb_pkt_out* d_recs, fb_batch_stats* d_stats,
                       void* stream);
/* The same for dense records that did not come from this context's last parse (records routed from
 * other ranks, fb_route_records_dev; a host's own record buffer): max_n = a host bound of the count,
 * the count itself is d_stats->n_session on the device (min with max_n).  max_n = 0 is an update
 * call without records. */
int fb_flow_update_records_dev(fb_ctx* ctx, const fb_pkt_out* d_recs, uint32_t max_n, fb_batch_stats* d_stats,
                               void* stream);

/*
 * Batched process_parsed_packet (src/packets.rs:202-537) without the decode: canonical key,
 * originator, Local/Global filter, history char for each fb_parsed_pkt, stream-compacted into
 * d_out (class SESSION, input order).  A record with a protocol other than 6/17 or a family other
 * than 2/10 is classified DROP.  DEVICE pointers, asynchronous; follow with fb_flow_update_dev
 * for the session-table upsert.  d_class (n bytes) may be NULL; d_stats is required.
 */
int fb_process_parsed_dev(fb_ctx* ctx, const fb_parsed_pkt* d_in, uint32_t n, fb_pkt_out* d_out,
                          uint8_t* d_class, fb_batch_stats* d_stats, void* stream);
/* Host-memory variant of fb_process_parsed_dev followed by the session-table upsert when the
 * context has a flow table (new_sessions / updated_sessions filled).  Synchronous. */
int fb_process_parsed(fb_ctx* ctx, const fb_parsed_pkt* in, uint32_t n, fb_pkt_out* out,
                      uint32_t* n_out, uint8_t* cls, fb_batch_stats* stats, void* stream);

/* Device-resident parse + classify + flow upsert: fb_parse_classify_dev followed by
 * fb_flow_update_dev on the same stream (d_out is required: the update reads the records). */
int fb_process_dev(fb_ctx* ctx, const uint8_t* d_frames, uint64_t frames_bytes,
                   const uint32_t* d_offsets, uint32_t n, fb_pkt_out* d_out, fb_dns_out* d_dns,
                   uint8_t* d_class, fb_batch_stats* d_stats, void* stream);

/*
 * Segmented output (one wavefront-compacted segment per FB_SEG_FRAMES frames; no cross-segment
 * compaction, so the kernel streams with no inter-workgroup dependency).  Segment s holds the
 * frames [64s, 64s+64) and owns d_out records [64s, 64s+64) (3584 bytes):
 *   - its SESSION records, packet order, in records [64s, 64s + n_session(s))
 *   - its DNS side records (fb_dns_out, 16 B), packet order, the j-th at byte offset
 *     (s+1)*3584 - 16*(j+1) of d_out (packed at the segment's tail)
 *   - d_seg[s] = n_session(s) | n_dns(s) << 16; the other bytes are left unwritten.
 * d_out needs room for ceil(n/64)*64 records, d_seg for ceil(n/64) words.  Same classification,
 * record layout and stats as fb_parse_classify_dev (which compacts across the whole batch).
 * DEVICE pointers, asynchronous.  d_class may be NULL; d_stats is required.
 */
#define FB_SEG_FRAMES 64u
int fb_parse_classify_seg_dev(fb_ctx* ctx, const uint8_t* d_frames, uint64_t frames_bytes,
                              const uint32_t* d_offsets, uint32_t n, fb_pkt_out* d_out,
                              uint32_t* d_seg, uint8_t* d_class, fb_batch_stats* d_stats,
                              void* stream);
/*
 * Several segmented batches in ONE launch: the same results as fb_parse_classify_seg_dev called
 * once per batch (each batch its own frames, offsets, d_out, d_seg, d_class, d_stats), but the
 * kernel streams from one batch into the next without a launch boundary, so the per-launch
 * start-up (configuration load, the first offsets -> headers round trips) and the tail are paid
 * once.  `batches` is a HOST array of `count` (1..FB_MAX_SEG_BATCHES) descriptors holding DEVICE
 * pointers; each batch follows the fb_parse_classify_seg_dev rules.  Asynchronous.
 */
#define FB_MAX_SEG_BATCHES 32u
typedef struct fb_seg_batch {
    const uint8_t* d_frames;
    uint64_t frames_bytes;     /* < 4 GiB */
    const uint32_t* d_offsets; /* n + 1 entries */
    uint32_t n;
    uint32_t reserved;         /* 0 */
    fb_pkt_out* d_out;         /* ceil(n/64)*64 records */
    uint32_t* d_seg;           /* ceil(n/64) words */
    uint8_t* d_class;          /* n bytes, or NULL */
    fb_batch_stats* d_stats;   /* required */
} fb_seg_batch;                /* 64 bytes */
int fb_parse_classify_seg_batches_dev(fb_ctx* ctx, const fb_seg_batch* batches, uint32_t count, void* stream);

/* ---- resident queue-fed parse: one batch per call without a launch per batch ----------------
 * A capture loop that hands over one batch at a time (src/capture.rs:1036-1061 runs the pair per
 * packet; a GPU capture engine fills one device buffer at a time) pays a kernel launch per call
 * above: its prologue and the tail of the last segments.  fb_seg_queue_create launches ONE
 * resident parse kernel on an internal stream; fb_seg_queue_submit hands it a batch through a
 * ring in pinned host memory (no launch, no stream operation) and returns a ticket; the batch's
 * outputs (segmented layout and stats, exactly as fb_parse_classify_seg_dev writes them) are
 * complete once fb_seg_queue_query(ticket) returns FB_OK.  Not stream-ordered: the batch's frames
 * and offsets must be in device memory when it is submitted, and stay untouched (like its output
 * buffers) until its ticket completes.  The context's configuration is captured at create.  While
 * a queue lives its kernel holds two workgroups on every CU (every one must be resident: the grid is
 * sized by the occupancy query); what it leaves free -- the registers of a fifth wave per SIMD, a third
 * of the LDS -- runs copies and small kernels beside it, and a kernel that needs more of a CU waits
 * until fb_seg_queue_destroy.  One queue per device at a time (a second create fails with
 * FB_ERR_INVAL while the first lives).  A queue left idle for idle_ms (0 = 5,000 ms) stops itself,
 * and one whose blocks were not all running idle_ms after create (CUs held by other work) is
 * reported the same way: its calls then fail with FB_ERR_INTERNAL (destroy it, create a new one).
 * HARD RULES while a queue lives:
 *   - never hipFree / fb_dev_free device memory on its device: the free waits for the resident
 *     kernel (measured: a 1-MB hipFree waited 4.8 s, until the idle limit stopped the kernel, while
 *     hipMalloc, H2D and D2H copies did not wait) -- free only after fb_seg_queue_destroy;
 *   - one producer thread: submit / query / wait / destroy of one queue are not synchronised with
 *     each other (two concurrent submits would write the same ring slot and hand out one ticket);
 *   - at most FB_QUEUE_MAX_SUBMISSIONS batches over the queue's life (the kernel numbers batches in
 *     32 bits): the submit after that fails with FB_ERR_INVAL -- destroy the queue and create a new
 *     one (at ~24 us per 1M-frame batch that is ~28 h of continuous capture). */
#define FB_QUEUE_MAX_DEPTH 32u
#define FB_QUEUE_MAX_SUBMISSIONS (0xFFFFFFFFull - FB_QUEUE_MAX_DEPTH)
typedef struct fb_seg_queue fb_seg_queue;
fb_seg_queue* fb_seg_queue_create(fb_ctx* ctx, uint32_t depth /* 1..FB_QUEUE_MAX_DEPTH, 0 = 8 */, uint32_t idle_ms);
/* FB_QUEUE_SHARED: the kernel takes one workgroup on each of an eighth of the CUs (instead of two on
 * every CU), leaving the rest of the device to the session-table update kernels (K2's two 80-KB
 * workgroups need a CU's whole LDS), so a host can apply each completed batch to the context's
 * table (fb_flow_update_seg_dev on the batch's d_out / d_seg, on a stream of its own) while the
 * queue keeps parsing -- one batch per call WITH the upsert.  The update must then allocate nothing
 * (hipFree would wait for the queue): create the context with FB_CFG_FIXED_TABLE and
 * max_batch_packets >= the largest batch, and run no history / enrichment / export that grows
 * scratch while the queue lives. */
#define FB_QUEUE_SHARED 1u
fb_seg_queue* fb_seg_queue_create_ex(fb_ctx* ctx, uint32_t depth, uint32_t idle_ms, uint32_t flags);
/* Blocks only while `depth` batches are in flight (until the oldest of them completes). */
int fb_seg_queue_submit(fb_seg_queue* q, const fb_seg_batch* batch, uint64_t* ticket);
/* Lower this queue's submission limit below FB_QUEUE_MAX_SUBMISSIONS (tests of the limit; a host
 * that wants to recycle its queue earlier).  FB_ERR_INVAL if `limit` is above the maximum or below
 * the batches already submitted. */
int fb_seg_queue_set_limit(fb_seg_queue* q, uint64_t limit);
int fb_seg_queue_query(fb_seg_queue* q, uint64_t ticket); /* FB_OK done, 1 pending, < 0 error */
int fb_seg_queue_wait(fb_seg_queue* q, uint64_t ticket);  /* polls until done (no blocking wait) */
int fb_seg_queue_destroy(fb_seg_queue* q);                /* after the submitted batches complete */

/* Dense records from a segmented batch of n frames (d_seg_out / d_seg of the calls above): the
 * SESSION records into d_out and the DNS side records into d_dns, batch-wide packet order, as
 * fb_parse_classify_dev lays them out (either may be NULL).  The counts are those of the
 * segments (= n_session / n_dns of the batch's stats).  DEVICE pointers, asynchronous; one
 * compaction at a time per context (it uses context scratch). */
int fb_seg_compact_dev(fb_ctx* ctx, const fb_pkt_out* d_seg_out, const uint32_t* d_seg, uint32_t n,
                       fb_pkt_out* d_out, fb_dns_out* d_dns, void* stream);

/* fb_process_parsed_dev with segmented output (same segment layout; no DNS records). */
int fb_process_parsed_seg_dev(fb_ctx* ctx, const fb_parsed_pkt* d_in, uint32_t n,
                              fb_pkt_out* d_out, uint32_t* d_seg, uint8_t* d_class,
                              fb_batch_stats* d_stats, void* stream);
/* Flow-table upsert of the SESSION records of a segmented batch of n frames (d_out / d_seg of
 * fb_parse_classify_seg_dev or fb_process_parsed_seg_dev); new/updated ADDED into d_stats. */
int fb_flow_update_seg_dev(fb_ctx* ctx, const fb_pkt_out* d_out, const uint32_t* d_seg, uint32_t n,
                           fb_batch_stats* d_stats, void* stream);
/* fb_parse_classify_seg_dev followed by fb_flow_update_seg_dev on the same stream, with the same
 * results.  Prefer it when the records are only needed for the table: its parse also writes each
 * session record's table partition to context scratch, and its update's bucketing pass reads
 * those instead of re-reading and hashing the records (DESIGN.md §4 has the C4 timings). */
int fb_process_seg_dev(fb_ctx* ctx, const uint8_t* d_frames, uint64_t frames_bytes,
                       const uint32_t* d_offsets, uint32_t n, fb_pkt_out* d_out, uint32_t* d_seg,
                       uint8_t* d_class, fb_batch_stats* d_stats, void* stream);
/* Pipelined fb_process_seg_dev for a stream of batches (continuous capture): the parse of this
 * batch is ordered on `stream`, its table update runs on the context's own update stream after
 * it, and `stream` waits only for the update of the batch two calls back -- so each parse overlaps
 * the previous batch's update.  Same results as fb_process_seg_dev over the same batches.  The
 * parse's outputs (records, segment counts, stats' parse fields) are ordered on `stream` as usual;
 * the update's (new/updated sessions in d_stats, the table) only after fb_flow_join(ctx, stream).
 * d_out / d_seg / d_stats are read by the update until the call two batches later has been issued
 * (rotate two buffer sets: reusing the previous batch's buffers is allowed but waits for its
 * update, i.e. does not overlap).  Every other entry point that reads or writes the table (update,
 * export, count, clear, history, enrichment, the fused calls) joins the update stream itself. */
int fb_process_seg_async_dev(fb_ctx* ctx, const uint8_t* d_frames, uint64_t frames_bytes,
                             const uint32_t* d_offsets, uint32_t n, fb_pkt_out* d_out, uint32_t* d_seg,
                             uint8_t* d_class, fb_batch_stats* d_stats, void* stream);
/* Order `stream` after every table update fb_process_seg_async_dev has issued. */
int fb_flow_join(fb_ctx* ctx, void* stream);

/*
 * History characters of the LAST flow update on this context, grouped per flow: a stable sort of
 * that batch's TCP records (those with FB_META_HAS_FLAGS) by (flow slot, record order), i.e. for
 * every flow the characters it appended to its history string in this batch, in packet order
 * (src/packets.rs:187-198, 410-426).  d_hist[p] = fb_pkt_out.hist_char, d_hist_slot[p] = the
 * flow's fb_flow_rec.slot, for p < *d_n_hist (device u32).  Appending each run to the flow's
 * string, batch after batch, reproduces the reference's history.  Both arrays need room for the
 * last update's record slots: the n frames / packets of its batch (dense), ceil(n/64)*64
 * (segmented); slots past *d_n_hist are scratch.  The update's d_recs (and d_seg, d_stats) must
 * still be valid.  DEVICE pointers, asynchronous on `stream`.
 */
int fb_flow_history_dev(fb_ctx* ctx, uint8_t* d_hist, uint32_t* d_hist_slot, uint32_t* d_n_hist,
                        void* stream);

/* ---- new-session enrichment (src/packets.rs:429-485; ASN src/asn.rs:32-63 + src/asn_db.rs:144-166;
 *      blacklists src/blacklists.rs:205-260, 456-560) -------------------------------------------- */
/* One ASN range (Db's RecordInternal, src/asn_db.rs:47-54) with IPs in session_key word layout.
 * One table per family, sorted by (start, end) as Db::from_tsv leaves it (src/asn_db.rs:137);
 * `record` is the caller's index of (as_number, country, owner). */
typedef struct fb_asn_range {
    uint32_t start[4];
    uint32_t end[4];
    uint32_t as_number;
    uint32_t record;
    uint32_t reserved[2];
} fb_asn_range; /* 48 bytes */
/* One IpNet of blacklist `list` (< FB_MAX_BLACKLISTS): addr/prefix as parsed (the host bits of
 * addr are ignored, as IpNet::contains does); a plain IP is a /32 or /128 (src/blacklists.rs:128-135). */
typedef struct fb_cidr {
    uint32_t addr[4];
    uint32_t family; /* 2 / 10 */
    uint32_t prefix;
    uint32_t list;
    uint32_t reserved;
} fb_cidr; /* 32 bytes */
#define FB_MAX_BLACKLISTS 64u
int fb_set_asn_tables(fb_ctx* ctx, const fb_asn_range* v4, uint32_t n4, const fb_asn_range* v6, uint32_t n6);
int fb_set_blacklists(fb_ctx* ctx, const fb_cidr* nets, uint32_t n);
/* Batched get_asn + is_ip_blacklisted for arbitrary addresses: d_asn[i] = fb_asn_range.record of
 * Db::lookup (its exact binary search), -1 = None; d_lists[i] bit l = some range of blacklist l
 * contains the address.  Either output may be NULL.  DEVICE pointers, asynchronous. */
int fb_ip_lookup_dev(fb_ctx* ctx, const fb_ip* d_ips, uint32_t n, int32_t* d_asn, uint64_t* d_lists,
                     void* stream);
/* The per-new-session lookups of process_parsed_packet for the flows in the table. */
typedef struct fb_flow_enrich {
    uint32_t slot;           /* fb_flow_rec.slot                                                  */
    uint32_t flags;          /* FB_ENRICH_* (src/packets.rs:429-435)                               */
    int32_t src_asn;         /* record of get_asn(src_ip) when !is_local_src, else -1 (packets.rs:468-485) */
    int32_t dst_asn;
    uint64_t src_blacklists; /* lists containing src_ip when !is_local_src (blacklists.rs:545-556) */
    uint64_t dst_blacklists;
} fb_flow_enrich;            /* 32 bytes */
enum fb_enrich_bits {
    FB_ENRICH_LOCAL_SRC = 1u, /* is_lan_ip(key.src_ip) */
    FB_ENRICH_LOCAL_DST = 2u,
    FB_ENRICH_SELF_SRC = 4u,  /* own_ips.contains(key.src_ip) */
    FB_ENRICH_SELF_DST = 8u
};
/* Enrich every flow of the table (new_only = 0) or only those the last update call created
 * (new_only = 1: the reference does these lookups when it inserts a session).  Records in no
 * particular order; *d_n (device u64) receives the count.  DEVICE pointers, asynchronous. */
int fb_flow_enrich_dev(fb_ctx* ctx, uint32_t new_only, fb_flow_enrich* d_out, uint64_t cap, uint64_t* d_n,
                       void* stream);

/* ---- DNS divert parse (src/dns.rs:35-99: DnsPacket::parse of dns-parser 0.8.0, then the query /
 *      response bookkeeping) ------------------------------------------------------------------ */
#define FB_DNS_MAX_NAME 256u  /* bytes of the dotted first-question name kept per message */
#define FB_DNS_MAX_ADDRS 8u   /* A / AAAA answers kept per message */
enum fb_dns_status {          /* DnsPacket::parse outcome (dns_parser::Error variants) */
    FB_DNS_OK = 0,
    FB_DNS_HEADER_TOO_SHORT = 1,
    FB_DNS_UNEXPECTED_EOF = 2,
    FB_DNS_BAD_POINTER = 3,
    FB_DNS_UNKNOWN_LABEL_FORMAT = 4,
    FB_DNS_LABEL_NOT_ASCII = 5,
    FB_DNS_INVALID_QUERY_TYPE = 6,
    FB_DNS_INVALID_QUERY_CLASS = 7,
    FB_DNS_INVALID_TYPE = 8,
    FB_DNS_INVALID_CLASS = 9,
    FB_DNS_WRONG_RDATA_LENGTH = 10,
    FB_DNS_ADDITIONAL_OPT = 11
};
enum fb_dns_flags {
    FB_DNS_QUERY = 1u,            /* header.query (QR bit clear)                              */
    FB_DNS_HAS_QUESTION = 2u,     /* questions.get(0) is Some                                 */
    FB_DNS_REVERSE = 4u,          /* the first qname ends with .in-addr.arpa / .ip6.arpa      */
    FB_DNS_NAME_TRUNCATED = 8u,   /* the name is longer than FB_DNS_MAX_NAME - 1 bytes         */
    FB_DNS_ADDRS_TRUNCATED = 16u  /* more than FB_DNS_MAX_ADDRS A / AAAA answers              */
};
typedef struct fb_dns_msg {
    uint32_t pkt_index;  /* the frame (fb_dns_out.pkt_index)                          */
    uint16_t id;         /* header.id (the transaction id the bookkeeping keys on)   */
    uint8_t status;      /* fb_dns_status                                            */
    uint8_t flags;       /* fb_dns_flags                                             */
    uint16_t questions;  /* header counts                                            */
    uint16_t answers;
    uint16_t name_len;   /* bytes of names[i] (dotted, no terminator needed)         */
    uint8_t n_addrs;     /* A / AAAA answers in addrs[i * FB_DNS_MAX_ADDRS ..]        */
    uint8_t reserved;
} fb_dns_msg;            /* 16 bytes */
/* Parse the DNS payloads of a batch's DNS side records (fb_parse_classify_dev's d_dns) the way
 * DnsPacket::parse does, keeping what process_dns_packet uses: id, query bit, the first
 * question's name, the A / AAAA answers in order.  n = d_dns entries; with d_stats non-NULL only
 * the first d_stats->n_dns (read on the device) are parsed.  d_names: n * FB_DNS_MAX_NAME bytes,
 * 4-byte aligned (the name is written a dword at a time; bytes past name_len are unspecified),
 * d_addrs: n * FB_DNS_MAX_ADDRS fb_ip.  DEVICE pointers, asynchronous.  The ordered bookkeeping
 * (pending queries by id, resolutions) stays on the host: a few operations per DNS packet. */
int fb_dns_parse_dev(fb_ctx* ctx, const uint8_t* d_frames, uint64_t frames_bytes, const fb_dns_out* d_dns,
                     uint32_t n, const fb_batch_stats* d_stats, fb_dns_msg* d_msgs, char* d_names,
                     fb_ip* d_addrs, void* stream);

int fb_flow_count(fb_ctx* ctx, uint64_t* n_flows, void* stream); /* synchronous */
/* Copy every flow (slot order) to host memory; *n = flows written (<= cap). Synchronous. */
int fb_flow_export(fb_ctx* ctx, fb_flow_rec* out, uint64_t cap, uint64_t* n, void* stream);
/* Same, into DEVICE memory; *d_n (device u64) receives the count. Asynchronous. */
int fb_flow_export_dev(fb_ctx* ctx, fb_flow_rec* d_out, uint64_t cap, uint64_t* d_n,
                       void* stream);
/* get_sessions (src/capture.rs:1578-1612): the flows that pass `filter` (fb_filter) evaluated at
 * query time, as the reference does per SessionInfo: LOCAL_ONLY keeps is_local_session! (is_lan_ip
 * of both key addresses under the context's CURRENT LAN configuration, src/sessions.rs:660-672),
 * GLOBAL_ONLY keeps is_global_session!, ALL keeps everything (= fb_flow_export).  Slot order.
 * Host variant synchronous; the _dev variant asynchronous, *d_n (device u64) = flows written. */
int fb_flow_export_sessions(fb_ctx* ctx, uint32_t filter, fb_flow_rec* out, uint64_t cap, uint64_t* n,
                            void* stream);
int fb_flow_export_sessions_dev(fb_ctx* ctx, uint32_t filter, fb_flow_rec* d_out, uint64_t cap, uint64_t* d_n,
                                void* stream);
int fb_flow_clear(fb_ctx* ctx, void* stream); /* clear_all_sessions, src/capture.rs:396 */
/* Flow-table geometry and growth.  `generation` counts the growths since fb_create: each moves
 * flows to new slots (fb_flow_rec.slot, the history's flow ids), and fb_flow_slot_remap gives the
 * last growth's old -> new slot map (old capacity entries, 0xFFFFFFFF = empty) so a host that keys
 * per-flow state by slot can follow.  flows / max_partition are those the last completed update
 * reported (no device wait).  Synchronous. */
typedef struct fb_flow_table_info {
    uint64_t capacity;      /* slots */
    uint64_t partitions;    /* of 512 slots */
    uint64_t generation;    /* growths so far */
    uint64_t flows;         /* occupied slots after the last completed update */
    uint64_t max_partition; /* fullest partition then */
    uint64_t reserved[3];
} fb_flow_table_info;
int fb_flow_table_info_get(fb_ctx* ctx, fb_flow_table_info* info);
int fb_flow_slot_remap(fb_ctx* ctx, uint32_t* old_to_new, uint64_t cap, uint64_t* n);
/* The table's deterministic 64-bit key hash (the reference's DashMap uses SipHash with a random
 * per-process key, src/sessions.rs:23 + dashmap RandomState, so it has no reproducible hash). */
uint64_t fb_flow_hash(const fb_session_key* key);

/* Every flow's fb_flow_time (timed contexts), with its table slot (join with fb_flow_rec.slot of an
 * export: the orders differ).  Device form: asynchronous, *d_n = records; host form: synchronous. */
int fb_flow_export_times_dev(fb_ctx* ctx, fb_flow_time* d_out, uint64_t cap, uint64_t* d_n, void* stream);
int fb_flow_export_times(fb_ctx* ctx, fb_flow_time* out, uint64_t cap, uint64_t* n, void* stream);

/* ---- multi-GPU session table (BASELINE configs[4]) ------------------------------
 * The reference runs one capture task per interface into ONE shared DashMap (src/capture.rs:946-1016,
 * src/packets.rs:329-535); W ranks that each parse a contiguous packet-index shard into their own
 * table merge them into that one table:
 *   1. every rank exports its table with fb_flow_export_merge_dev: records grouped by owner rank
 *      (the key's fb_flow_hash high word scaled to [0, world)), d_counts[world] = group sizes;
 *   2. all-to-all of the groups (RCCL), each owner receiving every rank's group in rank order;
 *   3. the owner merges them with fb_flow_merge_dev: one fb_flow_rec per key;
 *   4. all-gather of the owners' merged records.
 * The result equals the table ONE context builds from the same packets in global order (call k of
 * every rank = its shard of global batch k; global batch k is the ranks' shards in rank order) --
 * integer sums (segment_count too), MIN first_seen / end_seen, MAX last_seen, hist_len SUM,
 * hist_mask OR, in_segment and session flags from the records holding the key's latest / earliest
 * packet -- and conn_state / end_mask re-decided at the global first FIN/RST: the ending rank's
 * end_mask OR the S s H h of the other ranks that precede it (their first occurrence in an earlier
 * call, or in the same call on a lower rank).  Exact for any number of update calls per rank.  The
 * shard layout: global batch k is split into contiguous packet-index ranges, rank r's before rank
 * r+1's.  fb_flow_export_merge_dev takes the layout of equal shards of equal-size batches -- call k
 * of every rank is its shard of global batch k, starting at the same index `shard_first` in each --
 * and makes positions (k << 32) | (shard_first + pkt_index).  fb_flow_export_merge_map_dev takes
 * any layout -- unequal per-call batches, a short tail batch, a rank that makes no call for a batch
 * whose shard is empty -- as a call map: call_map[k] = (global batch of this rank's update call k)
 * << 32 | (global index of that shard's first packet), global batches increasing with k; positions
 * become (call_map[k] >> 32) << 32 | ((call_map[k] & 0xFFFFFFFF) + pkt_index) and char_call the
 * global batch numbers. */
typedef struct fb_flow_mrec {
    fb_flow_rec rec;        /* positions global; rec.slot = the exporting rank                    */
    uint32_t char_call[4];  /* update call of the flow's first S, s, H, h (FB_CALL_NONE: none)     */
} fb_flow_mrec;             /* 152 bytes */
/* Every flow of the table, grouped by owner rank (slot order inside a group), into d_out (room for
 * cap records); d_counts: `world` device u64 group sizes.  1 <= world <= 64, rank < world.
 * DEVICE pointers, asynchronous. */
int fb_flow_export_merge_dev(fb_ctx* ctx, uint32_t world, uint32_t rank, uint64_t shard_first, fb_flow_mrec* d_out,
                             uint64_t cap, uint64_t* d_counts, void* stream);
/* The same with a host call map (n_calls >= the context's update calls since create / clear; the
 * map is copied before the call returns). */
int fb_flow_export_merge_map_dev(fb_ctx* ctx, uint32_t world, uint32_t rank, const uint64_t* call_map, uint32_t n_calls,
                                 fb_flow_mrec* d_out, uint64_t cap, uint64_t* d_counts, void* stream);
/* Merge n records received by one owner (each rank's group, in rank order; a key at most once per
 * rank) into one fb_flow_rec per key (slot 0), in the order of each key's first record; *d_n
 * (device u64) = keys.  d_out: room for n records.  DEVICE pointers, asynchronous. */
int fb_flow_merge_dev(fb_ctx* ctx, const fb_flow_mrec* d_in, uint64_t n, fb_flow_rec* d_out, uint64_t* d_n,
                      void* stream);
/* Routed global table (every kind of session state exact, the capture-time state of timed contexts
 * included): instead of merging per-rank tables, each rank parses its shard (fb_parse_classify_dev,
 * no update) and routes every SESSION record to the owner of its key BEFORE the update; the owner
 * then runs ONE update call per global batch over what it received -- every rank's group in rank
 * order, i.e. the flow's packets in global order -- so its table is exactly the single-table state of
 * its flows (history, conn_state, timeouts).  This groups a rank's n_session (*d_stats, at most max_n)
 * dense records by owner (stable), makes pkt_index global (+ shard_first: the index of the shard's
 * first frame in the global batch), and with d_ts (the shard's frame times) writes each record's
 * capture time to d_ts_out beside it; d_counts[world] = group sizes.  The host moves the groups
 * (all-to-all), scatters the received times into a global-batch-sized array by pkt_index for
 * fb_set_frame_times, and calls fb_flow_update_records_dev on the received records (with a stats
 * struct whose n_session is their count; an owner that received none still makes the call, so update
 * calls stay global batches).  DEVICE pointers, asynchronous. */
int fb_route_records_dev(fb_ctx* ctx, const fb_pkt_out* d_recs, const fb_batch_stats* d_stats, uint32_t max_n,
                         uint32_t world, uint64_t shard_first, const uint64_t* d_ts, fb_pkt_out* d_out,
                         uint64_t* d_ts_out, uint64_t* d_counts, void* stream);
/* The owner rank fb_flow_export_merge_dev assigns a key to. */
uint32_t fb_flow_owner(const fb_session_key* key, uint32_t world);

/* ---- host ingest ring (replaces the reader thread -> Vec<u8> -> mpsc(1000) -> processor path,
 *      src/capture.rs:1016, 1082-1142, 1183-1249) ---------------------------------------------
 * The producer (capture callback) appends frames to the current batch of a ring of pinned host
 * batches; a full batch is submitted as H2D (copy stream) -> fb_process_dev (parse + classify +
 * session-table upsert, or fb_parse_classify_dev with FB_RING_NO_FLOW) -> batch stats back, while
 * the producer fills the next one.  With every batch in flight the producer waits for the oldest
 * (no drop-on-full).  The session table stays in HBM (fb_flow_export); DNS side records come back
 * with their payload bytes (fb_ring_poll_dns).  One producer thread per ring, one ring per ctx. */
typedef struct fb_ring fb_ring;
typedef struct fb_ring_config {
    uint32_t slots;       /* pinned batches, 2..64 (0 = 4)                       */
    uint32_t max_packets; /* frames per batch                                    */
    uint64_t max_bytes;   /* frame bytes per batch, < 4 GiB                      */
    uint32_t flags;       /* FB_RING_*                                           */
    uint32_t copy_threads; /* threads of fb_ring_push_block's copy into the pinned batch (the
                              producer + copy_threads - 1 helpers the ring owns; 0 or 1 = the
                              producer alone; at most 64); other calls are unaffected */
} fb_ring_config;
#define FB_RING_NO_FLOW 1u /* parse + classify only, no session-table update */
typedef struct fb_ring_dns {
    uint64_t packet_seq;     /* frames pushed into the ring before this one          */
    uint64_t payload_offset; /* into the payload buffer of fb_ring_poll_dns          */
    uint32_t payload_length;
    uint8_t protocol;        /* 6 / 17 */
    uint8_t family;          /* 2 / 10 */
    uint16_t reserved;
} fb_ring_dns; /* 24 bytes */
fb_ring* fb_ring_create(fb_ctx* ctx, const fb_ring_config* cfg); /* NULL on failure */
int fb_ring_destroy(fb_ring* r);
int fb_ring_push(fb_ring* r, const uint8_t* frame, uint32_t caplen);            /* copies one frame */
int fb_ring_push_block(fb_ring* r, const uint8_t* frames, const uint32_t* offsets, uint32_t n);
uint8_t* fb_ring_reserve(fb_ring* r, uint32_t caplen); /* zero-copy: write the frame there before the
                                                           next push/reserve/submit; NULL on error */
/* Zero-copy block for bulk producers (TPACKET_V3 blocks, capture engines): room for n frames of
 * `bytes` in total in one batch.  The caller writes the frames at the returned pointer and
 * offsets[k] = *base + (start of frame k within that area), k < n, before the next ring call. */
uint8_t* fb_ring_reserve_block(fb_ring* r, uint32_t n, uint64_t bytes, uint32_t** offsets, uint32_t* base);
int fb_ring_submit(fb_ring* r);                        /* submit the partly filled batch now      */
int fb_ring_sync(fb_ring* r);                          /* submit + wait for every batch           */
/* Totals over the completed batches (fields summed, error OR-ed), batches completed, frames pushed. */
int fb_ring_stats(fb_ring* r, fb_batch_stats* total, uint64_t* batches, uint64_t* frames);
/* Dequeue DNS side records of completed batches, their payloads packed into `payload`. */
int fb_ring_poll_dns(fb_ring* r, fb_ring_dns* out, uint32_t cap, uint8_t* payload, uint64_t payload_cap,
                     uint32_t* n, uint64_t* n_bytes);

/* ---- small device-memory helpers (so hosts without a GPU runtime binding can drive the
 *      device-resident entry points, e.g. through ctypes) ------------------------------- */
int fb_dev_alloc(void** p, uint64_t bytes);
int fb_dev_free(void* p);
int fb_host_alloc_pinned(void** p, uint64_t bytes);
int fb_host_free_pinned(void* p);
int fb_memcpy_h2d(void* dst, const void* src, uint64_t bytes, void* stream); /* async */
int fb_memcpy_d2h(void* dst, const void* src, uint64_t bytes, void* stream); /* async */
int fb_memset_dev(void* dst, int value, uint64_t bytes, void* stream);       /* async */
int fb_stream_create(void** stream);
int fb_stream_destroy(void* stream);
int fb_stream_sync(void* stream);
int fb_event_create(void** ev);
int fb_event_destroy(void* ev);
int fb_event_record(void* ev, void* stream);
int fb_event_elapsed_ms(float* ms, void* ev_start, void* ev_stop); /* syncs ev_stop */
int fb_event_query(void* ev); /* FB_OK once the event completed, 1 while pending: a capture loop
                                 polls it instead of blocking (no wake-up latency)          */
/* Busy-wait until the event completed: the polled completion without a call per poll. */
int fb_event_spin(void* ev);
int fb_device_count(int* n);
int fb_set_device(int device);
int fb_ctx_device(const fb_ctx* ctx, int* device); /* the device fb_create bound the context to */

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* FLODBADD_GPU_H */
