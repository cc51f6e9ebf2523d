//! Raw declarations of `include/iris_hip.h`, the C ABI of `libiris_hip.so`.
//!
//! One `extern "C"` item per function of the header, same names, same argument
//! order and C types (`tests/test_rust_binding.py` checks this file against the
//! header on every CPU test run, since this image has no Rust toolchain).
//! Every function returns an `int` status (`IRIS_OK` = 0) and leaves the message
//! of a failure in `iris_last_error()` (thread-local).
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int, c_void};

/// Geometry (src/lib.rs:10-12, src/bits.rs:10).
pub const IRIS_COLS: usize = 200;
pub const IRIS_ROWS: usize = 64;
pub const IRIS_BITS: usize = 12800;
pub const IRIS_LIMBS: usize = 200;
pub const IRIS_ROTATIONS: usize = 31;
pub const IRIS_MAX_ROTATION: i32 = 15;

/// Status codes.
pub const IRIS_OK: c_int = 0;
pub const IRIS_E_ARG: c_int = -1;
pub const IRIS_E_HIP: c_int = -2;
pub const IRIS_E_NOMEM: c_int = -3;
pub const IRIS_E_NODEV: c_int = -4;
pub const IRIS_E_RANGE: c_int = -5;
pub const IRIS_E_IO: c_int = -6;
pub const IRIS_E_FORMAT: c_int = -7;

/// Database record kinds.
pub const IRIS_KIND_MASKS: c_int = 1;
pub const IRIS_KIND_SHARES: c_int = 2;
pub const IRIS_KIND_TEMPLATES: c_int = 3;

/// Device layouts.
pub const IRIS_LAYOUT_DEFAULT: c_int = 0;
pub const IRIS_LAYOUT_LANES: c_int = 1;
pub const IRIS_LAYOUT_TILES: c_int = 2;

/// Bytes of a device group's RCCL id (`iris_group_unique_id`).
pub const IRIS_GROUP_ID_BYTES: usize = 128;
pub const IRIS_GROUP_BUS_ID_BYTES: usize = 32;

/// Opaque handles (`iris_device_t`, `iris_db_t`, `iris_engine_t`, `iris_pending_t`).
#[repr(C)]
pub struct IrisDevice {
    _private: [u8; 0],
}
#[repr(C)]
pub struct IrisDb {
    _private: [u8; 0],
}
#[repr(C)]
pub struct IrisEngine {
    _private: [u8; 0],
}
#[repr(C)]
pub struct IrisPending {
    _private: [u8; 0],
}
/// Device groups (`iris_group_t`, `iris_group_db_t`, `iris_group_pending_t`).
#[repr(C)]
pub struct IrisGroup {
    _private: [u8; 0],
}
#[repr(C)]
pub struct IrisGroupDb {
    _private: [u8; 0],
}
#[repr(C)]
pub struct IrisGroupPending {
    _private: [u8; 0],
}

/// `iris_template_t`: the reference's `#[repr(C)] Template { pattern, mask }`
/// (src/template.rs:11-29).
#[repr(C)]
#[derive(Clone, Copy)]
pub struct IrisTemplate {
    pub pattern: [u64; IRIS_LIMBS],
    pub mask: [u64; IRIS_LIMBS],
}

/// `iris_match_t`: the resolver's `(min_distance, min_index)` (src/main.rs:581-582,
/// 616-621) plus the exact fraction behind it.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq)]
pub struct IrisMatch {
    pub distance: f64,
    pub index: u64,
    pub num: u32,
    pub den: u32,
    pub rotation: i32,
    pub reserved: u32,
}

extern "C" {
    // errors
    pub fn iris_last_error() -> *const c_char;
    pub fn iris_version() -> *const c_char;
    pub fn iris_config(dev: *const IrisDevice, buf: *mut c_char, len: usize, needed: *mut usize) -> c_int;

    // devices
    pub fn iris_device_count(count: *mut c_int) -> c_int;
    pub fn iris_device_open(ordinal: c_int, out: *mut *mut IrisDevice) -> c_int;
    pub fn iris_device_close(dev: *mut IrisDevice) -> c_int;
    pub fn iris_device_synchronize(dev: *mut IrisDevice) -> c_int;
    pub fn iris_device_stream(dev: *mut IrisDevice, stream: *mut *mut c_void) -> c_int;
    pub fn iris_device_memory(dev: *mut IrisDevice, free_bytes: *mut usize, total_bytes: *mut usize) -> c_int;
    pub fn iris_device_set_profiling(dev: *mut IrisDevice, enabled: c_int) -> c_int;
    pub fn iris_device_kernel_stats(
        dev: *mut IrisDevice,
        kernel: *const c_char,
        launches: *mut u64,
        total_ms: *mut f64,
        items: *mut u64,
    ) -> c_int;
    pub fn iris_device_kernel_stats_largest(
        dev: *mut IrisDevice,
        kernel: *const c_char,
        items: *mut u64,
        ms: *mut f64,
    ) -> c_int;
    pub fn iris_device_reset_stats(dev: *mut IrisDevice) -> c_int;
    pub fn iris_device_alloc(dev: *mut IrisDevice, bytes: usize, ptr: *mut *mut c_void) -> c_int;
    pub fn iris_device_free(dev: *mut IrisDevice, ptr: *mut c_void) -> c_int;
    pub fn iris_device_drop_resident(dev: *mut IrisDevice) -> c_int;
    pub fn iris_device_drop_resident_range(dev: *mut IrisDevice, ptr: *const c_void) -> c_int;
    pub fn iris_memcpy_d2h(dev: *mut IrisDevice, host: *mut c_void, device: *const c_void, bytes: usize) -> c_int;
    pub fn iris_memcpy_h2d(dev: *mut IrisDevice, device: *mut c_void, host: *const c_void, bytes: usize) -> c_int;

    // databases
    pub fn iris_db_create(dev: *mut IrisDevice, kind: c_int, capacity: u64, out: *mut *mut IrisDb) -> c_int;
    pub fn iris_db_create_ex(
        dev: *mut IrisDevice,
        kind: c_int,
        capacity: u64,
        layout: c_int,
        out: *mut *mut IrisDb,
    ) -> c_int;
    pub fn iris_db_layout(db: *const IrisDb, layout: *mut c_int) -> c_int;
    pub fn iris_db_destroy(db: *mut IrisDb) -> c_int;
    pub fn iris_db_len(db: *const IrisDb, len: *mut u64) -> c_int;
    pub fn iris_db_capacity(db: *const IrisDb, cap: *mut u64) -> c_int;
    pub fn iris_db_kind(db: *const IrisDb, kind: *mut c_int) -> c_int;
    pub fn iris_db_append(db: *mut IrisDb, records: *const c_void, n: u64) -> c_int;
    pub fn iris_db_write(db: *mut IrisDb, index: u64, records: *const c_void, n: u64) -> c_int;
    pub fn iris_db_read(db: *const IrisDb, first: u64, n: u64, records: *mut c_void) -> c_int;
    pub fn iris_db_generate(db: *mut IrisDb, n: u64, seed: u64, global_index0: u64) -> c_int;
    pub fn iris_db_clear(db: *mut IrisDb) -> c_int;
    pub fn iris_db_truncate(db: *mut IrisDb, len: u64) -> c_int;

    // host residency
    pub fn iris_db_attach_host(db: *mut IrisDb, host: *const c_void, n: u64, upload: c_int) -> c_int;
    pub fn iris_db_detach_host(db: *mut IrisDb) -> c_int;

    // on-disk formats
    pub fn iris_db_load_file(db: *mut IrisDb, path: *const c_char, first: u64, count: u64, loaded: *mut u64)
        -> c_int;
    pub fn iris_db_save_file(db: *const IrisDb, path: *const c_char, first: u64, n: u64) -> c_int;
    pub fn iris_templates_read_json(path: *const c_char, out: *mut IrisTemplate, cap: u64, n: *mut u64) -> c_int;
    pub fn iris_templates_write_json(path: *const c_char, templates: *const IrisTemplate, n: u64) -> c_int;

    // share preparation
    pub fn iris_prepare_shares(
        templates: *const IrisDb,
        first: u64,
        n: u64,
        index_base: u64,
        key: *const [u8; 32],
        nonce: u64,
        rounds: u32,
        parties: u32,
        shares: *const *mut IrisDb,
        masks: *mut IrisDb,
    ) -> c_int;

    // engines
    pub fn iris_masks_engine_new(dev: *mut IrisDevice, query_mask: *const u64, out: *mut *mut IrisEngine) -> c_int;
    pub fn iris_distance_engine_new(dev: *mut IrisDevice, query: *const u16, out: *mut *mut IrisEngine) -> c_int;
    pub fn iris_template_engine_new(
        dev: *mut IrisDevice,
        query: *const IrisTemplate,
        out: *mut *mut IrisEngine,
    ) -> c_int;
    pub fn iris_engine_destroy(engine: *mut IrisEngine) -> c_int;
    pub fn iris_engine_batch_process(
        engine: *mut IrisEngine,
        db: *const IrisDb,
        first: u64,
        n: u64,
        out: *mut u16,
    ) -> c_int;
    pub fn iris_engine_batch_process_device(
        engine: *mut IrisEngine,
        db: *const IrisDb,
        first: u64,
        n: u64,
        out_device: *mut u16,
    ) -> c_int;
    pub fn iris_engine_batch_process_host(engine: *mut IrisEngine, db: *const c_void, n: u64, out: *mut u16)
        -> c_int;
    pub fn iris_template_counts(
        engine: *mut IrisEngine,
        db: *const IrisDb,
        first: u64,
        n: u64,
        num_out: *mut u16,
        den_out: *mut u16,
    ) -> c_int;
    pub fn iris_template_distances(
        engine: *mut IrisEngine,
        db: *const IrisDb,
        first: u64,
        n: u64,
        out: *mut f64,
    ) -> c_int;
    pub fn iris_template_search(
        engine: *mut IrisEngine,
        db: *const IrisDb,
        first: u64,
        n: u64,
        index_base: u64,
        dist_out_device: *mut f64,
        out: *mut IrisMatch,
    ) -> c_int;
    pub fn iris_template_search_async(
        engine: *mut IrisEngine,
        db: *const IrisDb,
        first: u64,
        n: u64,
        index_base: u64,
        out: *mut *mut IrisPending,
    ) -> c_int;
    pub fn iris_pending_wait(pending: *mut IrisPending, out: *mut IrisMatch) -> c_int;
    pub fn iris_template_batch_engine_new(
        dev: *mut IrisDevice,
        queries: *const IrisTemplate,
        nq: u32,
        out: *mut *mut IrisEngine,
    ) -> c_int;
    pub fn iris_template_batch_search(
        engine: *mut IrisEngine,
        db: *const IrisDb,
        first: u64,
        n: u64,
        index_base: u64,
        out: *mut IrisMatch,
    ) -> c_int;

    // resolver
    pub fn iris_resolver_search(
        dev: *mut IrisDevice,
        shares_device: *const *const u16,
        parts: u32,
        denoms_device: *const u16,
        n: u64,
        index_base: u64,
        dist_out_device: *mut f64,
        out: *mut IrisMatch,
    ) -> c_int;
    pub fn iris_resolver_search_masks(
        engine: *mut IrisEngine,
        masks_db: *const IrisDb,
        first: u64,
        n: u64,
        shares_device: *const *const u16,
        parts: u32,
        index_base: u64,
        dist_out_device: *mut f64,
        out: *mut IrisMatch,
    ) -> c_int;
    pub fn iris_resolver_search_masks_host(
        engine: *mut IrisEngine,
        masks_db: *const IrisDb,
        first: u64,
        n: u64,
        shares: *const *const u16,
        parts: u32,
        index_base: u64,
        out: *mut IrisMatch,
    ) -> c_int;
    pub fn iris_resolver_search_host(
        dev: *mut IrisDevice,
        shares: *const *const u16,
        parts: u32,
        denoms: *const u16,
        n: u64,
        index_base: u64,
        out: *mut IrisMatch,
    ) -> c_int;

    // arch plugin (batched all-pairs)
    pub fn iris_dot_bool_batch(
        dev: *mut IrisDevice,
        a: *const u64,
        na: u64,
        b: *const u64,
        nb: u64,
        out: *mut u16,
    ) -> c_int;
    pub fn iris_dot_u16_batch(
        dev: *mut IrisDevice,
        a: *const u16,
        na: u64,
        b: *const u16,
        nb: u64,
        out: *mut u16,
    ) -> c_int;

    // host-side value helpers
    pub fn iris_bits_rotated(input: *const u64, amount: i32, out: *mut u64) -> c_int;
    pub fn iris_encoded_rotated(input: *const u16, amount: i32, out: *mut u16) -> c_int;
    pub fn iris_encode(t: *const IrisTemplate, out: *mut u16) -> c_int;
    pub fn iris_decode_distance(distances: *const u16, denominators: *const u16, out: *mut f64) -> c_int;
    pub fn iris_query_table_sizes(kind: c_int, nq: u32, tab_bytes: *mut usize, frag_bytes: *mut usize) -> c_int;
    pub fn iris_engine_query_tables(
        engine: *const IrisEngine,
        tab: *mut c_void,
        tab_bytes: usize,
        frag: *mut c_void,
        frag_bytes: usize,
    ) -> c_int;
    pub fn iris_host_query_tables(
        kind: c_int,
        query: *const c_void,
        nq: u32,
        tab: *mut c_void,
        tab_bytes: usize,
        frag: *mut c_void,
        frag_bytes: usize,
    ) -> c_int;
    pub fn iris_match_merge(records: *const IrisMatch, count: u64, out: *mut IrisMatch) -> c_int;

    // device groups (multi-GPU)
    pub fn iris_group_create(ordinals: *const c_int, n: u32, out: *mut *mut IrisGroup) -> c_int;
    pub fn iris_group_unique_id(id: *mut u8) -> c_int;
    pub fn iris_group_create_rank(
        ordinal: c_int,
        nranks: u32,
        rank: u32,
        id: *const u8,
        out: *mut *mut IrisGroup,
    ) -> c_int;
    pub fn iris_group_destroy(group: *mut IrisGroup) -> c_int;
    pub fn iris_group_set_timeout(group: *mut IrisGroup, ms: u32) -> c_int;
    pub fn iris_group_info(
        group: *const IrisGroup,
        local_devices: *mut u32,
        ranks: *mut u32,
        first_rank: *mut u32,
    ) -> c_int;
    pub fn iris_group_rccl_info(group: *const IrisGroup, comm_ranks: *mut u32, bus_ids: *mut c_char, len: usize) -> c_int;
    pub fn iris_group_device(group: *const IrisGroup, i: u32, dev: *mut *mut IrisDevice) -> c_int;
    pub fn iris_group_db_create(
        group: *mut IrisGroup,
        kind: c_int,
        total: u64,
        layout: c_int,
        shards_per_device: u32,
        out: *mut *mut IrisGroupDb,
    ) -> c_int;
    pub fn iris_group_db_destroy(gdb: *mut IrisGroupDb) -> c_int;
    pub fn iris_group_db_info(
        gdb: *const IrisGroupDb,
        total: *mut u64,
        shards: *mut u32,
        first_shard: *mut u32,
        local_shards: *mut u32,
    ) -> c_int;
    pub fn iris_group_db_shard(
        gdb: *const IrisGroupDb,
        i: u32,
        db: *mut *mut IrisDb,
        first: *mut u64,
        count: *mut u64,
    ) -> c_int;
    pub fn iris_group_db_generate(gdb: *mut IrisGroupDb, seed: u64) -> c_int;
    pub fn iris_group_db_write(gdb: *mut IrisGroupDb, index: u64, records: *const c_void, n: u64) -> c_int;
    pub fn iris_group_db_read(gdb: *const IrisGroupDb, index: u64, n: u64, records: *mut c_void) -> c_int;
    pub fn iris_group_db_load_file(gdb: *mut IrisGroupDb, path: *const c_char, first: u64) -> c_int;
    pub fn iris_group_template_search(gdb: *mut IrisGroupDb, query: *const IrisTemplate, out: *mut IrisMatch)
        -> c_int;
    pub fn iris_group_template_search_async(
        gdb: *mut IrisGroupDb,
        query: *const IrisTemplate,
        out: *mut *mut IrisGroupPending,
    ) -> c_int;
    pub fn iris_group_pending_wait(pending: *mut IrisGroupPending, out: *mut IrisMatch) -> c_int;
    pub fn iris_group_template_batch_search(
        gdb: *mut IrisGroupDb,
        queries: *const IrisTemplate,
        nq: u32,
        out: *mut IrisMatch,
    ) -> c_int;
}
