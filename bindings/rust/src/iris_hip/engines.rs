//! The reference's engine API (src/lib.rs:28-94) on the GPU, signatures unchanged:
//!
//! ```text
//! DistanceEngine::new(query: &EncodedBits) -> Self                               src/lib.rs:33
//! DistanceEngine::batch_process(&self, out: &mut [[u16; 31]], db: &[EncodedBits]) src/lib.rs:42
//! MasksEngine::new(query: &Bits) -> Self                                         src/lib.rs:60
//! MasksEngine::batch_process(&self, out: &mut [[u16; 31]], db: &[Bits])          src/lib.rs:69
//! distances(&EncodedBits, &EncodedBits) -> [u16; 31]                             src/lib.rs:82
//! denominators(&Bits, &Bits) -> [u16; 31]                                        src/lib.rs:89
//! ```
//!
//! With the `hip` feature, `src/lib.rs` re-exports these instead of its rayon engines
//!.  `new` builds the 31 rotated query copies once — on the device,
//! in the layouts the kernels read — as the reference builds them once on the host.
//! `batch_process` keeps the reference contract: host slices in, host `[u16; 31]`
//! rows out, blocking, `assert_eq!(out.len(), db.len())`.  The device-resident forms
//! (`*_resident`, `TemplateEngine::search`) are what a participant / resolver uses
//! once its share or masks file is loaded into a `Database`.
use std::ptr;

use super::{check, default_device, ffi, match_to_pair, Database, Device, Record, Result, ShardedDatabase};
use crate::{Bits, EncodedBits, Template};

/// An engine handle plus the device it lives on (kept alive by the clone).
struct Handle {
    raw: *mut ffi::IrisEngine,
    _device: Device,
}

unsafe impl Send for Handle {}
unsafe impl Sync for Handle {}

impl Drop for Handle {
    fn drop(&mut self) {
        unsafe {
            ffi::iris_engine_destroy(self.raw);
        }
    }
}

impl Handle {
    fn batch_process_host<T: Record>(&self, what: &str, out: &mut [[u16; 31]], db: &[T]) {
        assert_eq!(out.len(), db.len());
        if db.is_empty() {
            return;
        }
        check(unsafe {
            ffi::iris_engine_batch_process_host(self.raw, db.as_ptr().cast(), db.len() as u64, out.as_mut_ptr().cast())
        })
        .unwrap_or_else(|e| panic!("{what}::batch_process: {e}"));
    }

    fn batch_process_resident(&self, out: &mut [[u16; 31]], db: &Database, first: u64) -> Result<()> {
        check(unsafe {
            ffi::iris_engine_batch_process(self.raw, db.raw(), first, out.len() as u64, out.as_mut_ptr().cast())
        })
    }
}

/// `DistanceEngine` (src/lib.rs:28-53): out[i][k] = dot_u16(rot(query, k - 15), db[i]) mod 2^16.
pub struct DistanceEngine {
    h: Handle,
}

impl DistanceEngine {
    pub fn new(query: &EncodedBits) -> Self {
        Self::new_on(default_device(), query).unwrap_or_else(|e| panic!("DistanceEngine::new: {e}"))
    }

    pub fn new_on(device: &Device, query: &EncodedBits) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_distance_engine_new(device.raw(), query.0.as_ptr(), &mut raw) })?;
        Ok(Self { h: Handle { raw, _device: device.clone() } })
    }

    pub fn batch_process(&self, out: &mut [[u16; 31]], db: &[EncodedBits]) {
        self.h.batch_process_host("DistanceEngine", out, db)
    }

    /// Records [first, first + out.len()) of a resident share database.
    pub fn batch_process_resident(&self, out: &mut [[u16; 31]], db: &Database, first: u64) -> Result<()> {
        self.h.batch_process_resident(out, db, first)
    }
}

/// `MasksEngine` (src/lib.rs:55-80): out[i][k] = dot_bool(rot(query, k - 15), db[i]).
pub struct MasksEngine {
    h: Handle,
}

impl MasksEngine {
    pub fn new(query: &Bits) -> Self {
        Self::new_on(default_device(), query).unwrap_or_else(|e| panic!("MasksEngine::new: {e}"))
    }

    pub fn new_on(device: &Device, query: &Bits) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_masks_engine_new(device.raw(), query.0.as_ptr(), &mut raw) })?;
        Ok(Self { h: Handle { raw, _device: device.clone() } })
    }

    pub fn batch_process(&self, out: &mut [[u16; 31]], db: &[Bits]) {
        self.h.batch_process_host("MasksEngine", out, db)
    }

    pub fn batch_process_resident(&self, out: &mut [[u16; 31]], db: &Database, first: u64) -> Result<()> {
        self.h.batch_process_resident(out, db, first)
    }

    /// The resolver's step in one pass (src/main.rs:510-519 + 597-621): denominators of
    /// masks [first, first + n) from this engine, the wrapping sum of the participants'
    /// share rows (DEVICE arrays of n x 31 u16), decode and first strict minimum.
    pub fn resolve(&self, masks: &Database, first: u64, n: u64, shares_device: &[*const u16]) -> Result<(f64, usize)> {
        let mut m = ffi::IrisMatch::default();
        check(unsafe {
            ffi::iris_resolver_search_masks(
                self.h.raw,
                masks.raw(),
                first,
                n,
                shares_device.as_ptr(),
                shares_device.len() as u32,
                0,
                ptr::null_mut(),
                &mut m,
            )
        })?;
        Ok(match_to_pair(&m))
    }

    /// The same step with the participants' replies still in host memory (`shares[p]` holds the
    /// n = `shares[p].len()` rows of records [first, first + n)): the library sums the parts on
    /// the host and uploads only the sum (iris_resolver_search_masks_host).
    pub fn resolve_host(&self, masks: &Database, first: u64, shares: &[&[[u16; 31]]]) -> Result<(f64, usize)> {
        let n = shares.first().map_or(0, |s| s.len());
        assert!(shares.iter().all(|s| s.len() == n), "share arrays of different lengths");
        let ptrs: Vec<*const u16> = shares.iter().map(|s| s.as_ptr() as *const u16).collect();
        let mut m = ffi::IrisMatch::default();
        check(unsafe {
            ffi::iris_resolver_search_masks_host(
                self.h.raw,
                masks.raw(),
                first,
                n as u64,
                ptrs.as_ptr(),
                ptrs.len() as u32,
                0,
                &mut m,
            )
        })?;
        Ok(match_to_pair(&m))
    }
}

/// `distances` (src/lib.rs:82-87).
pub fn distances(query: &EncodedBits, entry: &EncodedBits) -> [u16; 31] {
    let mut result = [0_u16; 31];
    DistanceEngine::new(query).batch_process(std::slice::from_mut(&mut result), std::slice::from_ref(entry));
    result
}

/// `denominators` (src/lib.rs:89-94).
pub fn denominators(query: &Bits, entry: &Bits) -> [u16; 31] {
    let mut result = [0_u16; 31];
    MasksEngine::new(query).batch_process(std::slice::from_mut(&mut result), std::slice::from_ref(entry));
    result
}

/// Plaintext masked Hamming of one query against a resident Template database:
/// `Template::distance` per record (src/template.rs:43-64) and the resolver's
/// `(min_distance, min_index)` (src/main.rs:616-621), bit-exact.
pub struct TemplateEngine {
    h: Handle,
    query: Template,
}

/// An enqueued search (`iris_template_search_async`); `wait` blocks for it alone.
pub struct PendingSearch {
    raw: *mut ffi::IrisPending,
}

unsafe impl Send for PendingSearch {}

impl PendingSearch {
    pub fn wait(mut self) -> Result<(f64, usize)> {
        let mut m = ffi::IrisMatch::default();
        let raw = std::mem::replace(&mut self.raw, ptr::null_mut());
        check(unsafe { ffi::iris_pending_wait(raw, &mut m) })?;
        Ok(match_to_pair(&m))
    }
}

impl Drop for PendingSearch {
    fn drop(&mut self) {
        if !self.raw.is_null() {
            let mut m = ffi::IrisMatch::default();
            unsafe {
                ffi::iris_pending_wait(self.raw, &mut m);
            }
        }
    }
}

impl TemplateEngine {
    pub fn new(query: &Template) -> Self {
        Self::new_on(default_device(), query).unwrap_or_else(|e| panic!("TemplateEngine::new: {e}"))
    }

    pub fn new_on(device: &Device, query: &Template) -> Result<Self> {
        let mut raw = ptr::null_mut();
        let q = query as *const Template as *const ffi::IrisTemplate;
        check(unsafe { ffi::iris_template_engine_new(device.raw(), q, &mut raw) })?;
        Ok(Self { h: Handle { raw, _device: device.clone() }, query: *query })
    }

    /// The same query over a sharded multi-GPU database (every device builds its own
    /// engine, searches its shards; winners all-gathered over RCCL and merged).
    pub fn search_sharded(&self, db: &ShardedDatabase) -> Result<(f64, usize)> {
        db.search(&self.query)
    }

    /// `Template::distance(query, db[i])` for i in [first, first + out.len()).
    pub fn distances(&self, db: &Database, first: u64, out: &mut [f64]) -> Result<()> {
        check(unsafe { ffi::iris_template_distances(self.h.raw, db.raw(), first, out.len() as u64, out.as_mut_ptr()) })
    }

    /// Min / argmin over records [first, first + n); indices are `index_base + i`.
    pub fn search(&self, db: &Database, first: u64, n: u64, index_base: u64) -> Result<(f64, usize)> {
        let mut m = ffi::IrisMatch::default();
        check(unsafe {
            ffi::iris_template_search(self.h.raw, db.raw(), first, n, index_base, ptr::null_mut(), &mut m)
        })?;
        Ok(match_to_pair(&m))
    }

    /// Enqueues the search and returns at once (the engine may be dropped before the
    /// wait; the database must outlive it).
    pub fn search_async(&self, db: &Database, first: u64, n: u64, index_base: u64) -> Result<PendingSearch> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_template_search_async(self.h.raw, db.raw(), first, n, index_base, &mut raw) })?;
        Ok(PendingSearch { raw })
    }
}

#[cfg(test)]
mod tests {
    //! The reference's engine semantics against plain host loops (wrapping u16 MACs and
    //! popcounts over the reference's own rotations), on random records.
    use super::*;
    use rand::{thread_rng, Rng};

    #[test]
    fn distance_engine_matches_host_loop() {
        let mut rng = thread_rng();
        let q: EncodedBits = rng.gen();
        let db: Vec<EncodedBits> = (0..37).map(|_| rng.gen()).collect();
        let mut out = vec![[0u16; 31]; db.len()];
        DistanceEngine::new(&q).batch_process(&mut out, &db);
        for (row, e) in out.iter().zip(db.iter()) {
            for (k, &got) in row.iter().enumerate() {
                let r = q.rotated(k as i32 - 15);
                let want = r.0.iter().zip(e.0.iter()).fold(0u16, |s, (&a, &b)| s.wrapping_add(a.wrapping_mul(b)));
                assert_eq!(got, want);
            }
        }
    }

    #[test]
    fn masks_engine_matches_host_loop() {
        let mut rng = thread_rng();
        let q: Bits = rng.gen();
        let db: Vec<Bits> = (0..37).map(|_| rng.gen()).collect();
        let mut out = vec![[0u16; 31]; db.len()];
        MasksEngine::new(&q).batch_process(&mut out, &db);
        for (row, e) in out.iter().zip(db.iter()) {
            for (k, &got) in row.iter().enumerate() {
                let r = q.rotated(k as i32 - 15);
                let want: u32 = r.0.iter().zip(e.0.iter()).map(|(&a, &b)| (a & b).count_ones()).sum();
                assert_eq!(got as u32, want);
            }
        }
    }

    #[test]
    #[should_panic]
    fn batch_process_length_mismatch_panics() {
        let mut rng = thread_rng();
        let q: Bits = rng.gen();
        let db: Vec<Bits> = (0..3).map(|_| rng.gen()).collect();
        let mut out = vec![[0u16; 31]; 2];
        MasksEngine::new(&q).batch_process(&mut out, &db);
    }

    #[test]
    fn template_search_matches_template_distance() {
        let mut rng = thread_rng();
        let query: Template = rng.gen();
        let mut records: Vec<Template> = (0..100).map(|_| rng.gen()).collect();
        records[61] = query.rotated(7);
        let dev = default_device();
        let mut db = Database::new::<Template>(dev, records.len() as u64).unwrap();
        db.append(&records).unwrap();
        let engine = TemplateEngine::new(&query);
        let mut d = vec![0f64; records.len()];
        engine.distances(&db, 0, &mut d).unwrap();
        for (got, r) in d.iter().zip(records.iter()) {
            assert_eq!(got.to_bits(), query.distance(r).to_bits());
        }
        let (best, index) = engine.search(&db, 0, records.len() as u64, 0).unwrap();
        assert_eq!((best, index), (0.0, 61));
    }

    #[test]
    fn attached_slices_match_host_loop() {
        // the resolver's loop (src/main.rs:511-516) over an attached array: no upload per chunk
        let mut rng = thread_rng();
        let q: Bits = rng.gen();
        let masks: Vec<Bits> = (0..5000).map(|_| rng.gen()).collect();
        let att = crate::iris_hip::AttachedDatabase::new(default_device(), &masks).unwrap();
        let engine = MasksEngine::new(&q);
        for chunk in masks.chunks(1234) {
            let mut out = vec![[0u16; 31]; chunk.len()];
            engine.batch_process(&mut out, chunk);
            for (row, e) in out.iter().zip(chunk.iter()) {
                for (k, &got) in row.iter().enumerate() {
                    let r = q.rotated(k as i32 - 15);
                    let want: u32 = r.0.iter().zip(e.0.iter()).map(|(&a, &b)| (a & b).count_ones()).sum();
                    assert_eq!(got as u32, want);
                }
            }
        }
        drop(att);
    }

    #[test]
    fn sharded_search_matches_single_device() {
        let mut rng = thread_rng();
        let query: Template = rng.gen();
        let mut records: Vec<Template> = (0..1000).map(|_| rng.gen()).collect();
        records[777] = query.rotated(-4);
        let group = crate::iris_hip::Group::new(&[0]).unwrap();
        let mut sdb = ShardedDatabase::new(&group, records.len() as u64, ffi::IRIS_LAYOUT_DEFAULT, 4).unwrap();
        sdb.write(0, &records).unwrap();
        let engine = TemplateEngine::new(&query);
        assert_eq!(engine.search_sharded(&sdb).unwrap(), (0.0, 777));
    }
}
