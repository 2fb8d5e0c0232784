/*
 * oracle.h -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product path (flodbadd_amd/, libflodbadd_gpu.so) never links or calls it.
 *
 * Restates, from edamametechnologies/flodbadd @ 2025-07-18:
 *   src/packets.rs:603-802   parse_packet_pcap (via pnet_packet 0.35.0 semantics, which are
 *                            NOT vendored in the reference: byte-level decode parity is
 *                            "unpinned" -- see DESIGN.md §Oracle)
 *   src/packets.rs:202-537   process_parsed_packet (canonical key, originator, filter, upsert)
 *   src/packets.rs:105-200   update_session_stats (integer counters + history)
 *   src/packets.rs:539-601   determine_conn_state, map_tcp_flags
 *   src/ip.rs:55-242         is_lan_ip
 *   src/sessions.rs:658-692  is_local_session! / is_global_session! / filter_sessions
 *   src/port_vulns.rs:213-228 get_name_from_port (as a 65536-bit "has a name" bitmap)
 *   src/asn_db.rs:82-166     Db::from_tsv filtering/sort + Db::lookup (ASN)
 *   src/blacklists.rs:205-260 is_ip_in_blacklist (IpNet::contains scan)
 *   src/dns.rs:35-99         process_dns_packet's use of dns_parser::Packet::parse (dns-parser
 *                            0.8.0, NOT vendored: DNS parse parity is "unpinned" too)
 * Output records use the same C layout as include/flodbadd_gpu.h so results compare
 * byte-for-byte.
 */
#ifndef FLODBADD_ORACLE_H
#define FLODBADD_ORACLE_H

#include <stdint.h>
#include "../include/flodbadd_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Result kinds of parse_packet_pcap (Option<ParsedPacket>). */
enum orc_kind { ORC_NONE = 0, ORC_SESSION = 1, ORC_DNS = 2 };

/* SessionPacketData / DnsPacketData (src/packets.rs:85-102), flattened. */
typedef struct orc_parsed {
    uint32_t kind;
    uint8_t protocol; /* 6 / 17 */
    uint8_t family;   /* 2 / 10 */
    uint8_t has_flags;
    uint8_t flags;
    uint32_t src_ip[4], dst_ip[4]; /* session_key word format */
    uint16_t src_port, dst_port;
    uint32_t packet_length;
    uint32_t ip_packet_length;
    uint32_t dns_payload_offset; /* relative to the frame start */
    uint32_t dns_payload_length;
} orc_parsed;

typedef struct orc_cfg {
    uint32_t filter;
    uint8_t service_bitmap[FB_SERVICE_BITMAP_BYTES];
    uint32_t n_lan_v6;
    fb_lan_v6 lan_v6[FB_MAX_LAN_V6];
    uint32_t n_own_ips;
    fb_ip own_ips[FB_MAX_OWN_IPS];
} orc_cfg;

/* Single-frame decode. Returns kind. */
uint32_t orc_parse_packet_pcap(const uint8_t* frame, uint32_t caplen, orc_parsed* out);

int orc_is_service_port(const orc_cfg* cfg, uint16_t port);
int orc_is_lan_ip(const orc_cfg* cfg, uint32_t family, const uint32_t ip[4]);
char orc_map_tcp_flags(uint8_t flags, uint32_t packet_length, int is_originator);

/* Per-packet classification (the stateless part of process_parsed_packet).
 * Returns FB_CLASS_SESSION or FB_CLASS_FILTERED; fills *rec either way. */
uint32_t orc_classify(const orc_cfg* cfg, const orc_parsed* p, uint32_t pkt_index,
                      fb_pkt_out* rec);

/* Whole batch, same contract as fb_parse_classify (any output pointer may be NULL). */
int orc_parse_classify(const orc_cfg* cfg, const uint8_t* frames, uint64_t frames_bytes,
                       const uint32_t* offsets, uint32_t n, fb_pkt_out* out, uint32_t* n_out,
                       fb_dns_out* dns, uint32_t* n_dns, uint8_t* cls, fb_batch_stats* stats);

/* Batched process_parsed_packet (src/packets.rs:202-327) over fb_parsed_pkt records, same
 * contract as fb_process_parsed_dev: PACKET_STATS before the filter, SESSION records compacted
 * in input order, protocol not 6/17 or family not 2/10 -> DROP. */
int orc_process_parsed(const orc_cfg* cfg, const fb_parsed_pkt* in, uint32_t n, fb_pkt_out* out,
                       uint32_t* n_out, uint8_t* cls, fb_batch_stats* stats);

/* ---- session table (DashMap<Session, SessionInfo> restated; integer part + history) ---- */
typedef struct orc_flows orc_flows;
orc_flows* orc_flows_new(void);
void orc_flows_free(orc_flows* f);
void orc_flows_clear(orc_flows* f);
/* Upsert records in order; adds new/updated counts into stats (may be NULL). */
/* One call = one flow-table update (the high word of fb_flow_rec positions, FB_SEEN_NONE etc.). */
void orc_flows_update(orc_flows* f, const fb_pkt_out* recs, uint64_t n, fb_batch_stats* stats);
/* The same with capture timestamps (ts[pkt_index] ns): segment state with the 5-s timeout and the
 * capture-time fields of fb_flow_time (src/packets.rs:137-200, 352-426). */
void orc_flows_update_timed(orc_flows* f, const fb_pkt_out* recs, uint64_t n, fb_batch_stats* stats,
                            const uint64_t* ts);
/* fb_flow_time per flow in orc_flows_export_sorted order (slot 0); ref_f64 (optional, 2 per flow):
 * the reference's own f64 total_segment_interarrival and segment_interarrival. */
uint64_t orc_flows_export_times(const orc_flows* f, fb_flow_time* out, double* ref_f64, uint64_t cap);
uint64_t orc_flows_count(const orc_flows* f);
/* Export sorted by the derived Ord of Session (src/sessions.rs:23-30). Returns count. */
uint64_t orc_flows_export_sorted(const orc_flows* f, fb_flow_rec* out, uint64_t cap);
/* History string + conn_state ('\0' when None) of one flow; returns history length, or -1. */
int64_t orc_flows_history(const orc_flows* f, const fb_session_key* key, char* buf,
                          uint64_t cap, char* conn_state, uint64_t cs_cap);

/* Multi-GPU merge restated (fb_flow_export_merge_dev / fb_flow_merge_dev semantics, include/
 * flodbadd_gpu.h): the table's flows grouped by owner rank (Ord order inside a group), positions
 * global, rec.slot = rank; counts[world] = group sizes.  Returns the records written (the table's
 * flow count; `out` must hold it). */
uint64_t orc_flow_hash(const fb_session_key* key);
uint64_t orc_flows_export_merge(const orc_flows* f, uint32_t world, uint32_t rank, uint64_t shard_first,
                                fb_flow_mrec* out, uint64_t* counts);
/* The same under a call map (fb_flow_export_merge_map_dev): call_map[k] = global batch of update call
 * k << 32 | global index of that shard's first packet. */
uint64_t orc_flows_export_merge_map(const orc_flows* f, uint32_t world, uint32_t rank, const uint64_t* call_map,
                                    fb_flow_mrec* out, uint64_t* counts);
/* One owner's received records (rank order) -> one record per key, in the order of each key's first
 * record.  Returns the keys written (`out` must hold n). */
uint64_t orc_flow_merge(const fb_flow_mrec* in, uint64_t n, fb_flow_rec* out);

/* Bench helper: parse+classify+upsert with a scratch record buffer; returns packets done. */
/* ---- new-session enrichment (ASN src/asn_db.rs:82-166, blacklists src/blacklists.rs:205-260) ---- */
uint32_t orc_asn_prepare(fb_asn_range* recs, uint32_t n, uint32_t family);
int32_t orc_asn_lookup(const fb_asn_range* recs, uint32_t n, uint32_t family, const uint32_t ip[4]);
uint64_t orc_blacklist_mask(const fb_cidr* nets, uint32_t n, uint32_t family, const uint32_t ip[4]);
void orc_enrich_keys(const orc_cfg* c, const fb_asn_range* a4, uint32_t n4, const fb_asn_range* a6, uint32_t n6,
                     const fb_cidr* nets, uint32_t nn, const fb_session_key* keys, uint32_t nk,
                     fb_flow_enrich* out);

/* All-cores baseline: `threads` contiguous ranges in parallel (OpenMP), compacted in packet order. */
int orc_parse_classify_mt(const orc_cfg* cfg, const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                          uint32_t n, fb_pkt_out* out, uint32_t* n_out, fb_dns_out* dns, uint32_t* n_dns,
                          fb_batch_stats* stats, int threads);

/* ---- DNS divert parse (dns-parser 0.8.0 Packet::parse restated; src/dns.rs:35-99) ---- */
uint32_t orc_dns_parse(const uint8_t* payload, uint32_t len, uint32_t pkt_index, fb_dns_msg* r, char* name,
                       fb_ip* addrs);

uint64_t orc_pipeline(const orc_cfg* cfg, orc_flows* flows, const uint8_t* frames,
                      uint64_t frames_bytes, const uint32_t* offsets, uint32_t n,
                      fb_pkt_out* scratch, fb_batch_stats* stats);

/* All-cores C4 baseline: parse + classify in `threads` ranges, then each thread upserts the keys
 * it owns (by key hash) into tables[thread]; the union of the tables = the single-thread table. */
uint64_t orc_pipeline_mt(const orc_cfg* cfg, orc_flows** tables, int threads, const uint8_t* frames,
                         uint64_t frames_bytes, const uint32_t* offsets, uint32_t n, fb_pkt_out* scratch,
                         fb_dns_out* dns_scratch, fb_batch_stats* st);
/* Derived Ord comparison of two keys (protocol, src_ip, src_port, dst_ip, dst_port). */
int orc_key_cmp(const fb_session_key* a, const fb_session_key* b);

#ifdef __cplusplus
}
#endif
#endif
