//! Safe layer over `libiris_hip.so` (MI355X / gfx950 kernels behind the C ABI of
//! `include/iris_hip.h`), written as a module of the reference crate: drop
//! `src/iris_hip/` next to `src/arch/hip.rs` and enable the `hip` feature
//! (INTEGRATION.md lists the three lines that change in the crate).
//!
//! Ownership follows the C ABI: host buffers belong to the caller and are never
//! retained after a call returns; device memory belongs to the handles here and is
//! released on `Drop`.  Every handle keeps the `Device` it was created on alive.
//! Errors are `Result<_, Error>`; the reference-signature wrappers in `engines`
//! panic where the reference panics (`assert_eq!(out.len(), db.len())`,
//! src/lib.rs:43,70) and on device errors, since the reference API has no
//! `Result` to return.

pub mod engines;
pub mod ffi;

use std::{
    ffi::{CStr, CString},
    fmt,
    marker::PhantomData,
    os::raw::{c_int, c_void},
    path::Path,
    ptr,
    sync::{Arc, OnceLock},
};

use crate::{Bits, EncodedBits, Template};

/// A failed ABI call: the status code and `iris_last_error()`.
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct Error {
    pub code: i32,
    pub message: String,
}

impl fmt::Display for Error {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "iris_hip error {}: {}", self.code, self.message)
    }
}

impl std::error::Error for Error {}

pub type Result<T> = std::result::Result<T, Error>;

/// Turns an ABI status into a `Result`, reading the thread's last error message.
pub fn check(rc: c_int) -> Result<()> {
    if rc == ffi::IRIS_OK {
        return Ok(());
    }
    let message = unsafe {
        let p = ffi::iris_last_error();
        if p.is_null() {
            String::new()
        } else {
            CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    };
    Err(Error { code: rc, message })
}

struct DeviceInner(*mut ffi::IrisDevice);

// The library serialises calls per device internally (include/iris_hip.h, "Handles are
// thread-safe"), as the reference engines are `Sync` and shared by rayon workers.
unsafe impl Send for DeviceInner {}
unsafe impl Sync for DeviceInner {}

impl Drop for DeviceInner {
    fn drop(&mut self) {
        unsafe {
            ffi::iris_device_close(self.0);
        }
    }
}

/// One gfx950 device and its stream; cheap to clone (shared handle).
#[derive(Clone)]
pub struct Device(Arc<DeviceInner>);

impl Device {
    pub fn open(ordinal: i32) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_device_open(ordinal, &mut raw) })?;
        Ok(Device(Arc::new(DeviceInner(raw))))
    }

    pub fn count() -> Result<i32> {
        let mut n: c_int = 0;
        check(unsafe { ffi::iris_device_count(&mut n) })?;
        Ok(n)
    }

    pub fn raw(&self) -> *mut ffi::IrisDevice {
        self.0 .0
    }

    pub fn synchronize(&self) -> Result<()> {
        check(unsafe { ffi::iris_device_synchronize(self.raw()) })
    }

    /// (free, total) device memory in bytes.
    pub fn memory(&self) -> Result<(usize, usize)> {
        let (mut free, mut total) = (0usize, 0usize);
        check(unsafe { ffi::iris_device_memory(self.raw(), &mut free, &mut total) })?;
        Ok((free, total))
    }

    /// Frees the device's copy of the record file whose mapping holds `records` (the participant's
    /// or resolver's mmap'd slice): for a process that rewrites its file through a writable mapping,
    /// which the per-call staleness check does not see (iris_device_drop_resident_range).
    pub fn drop_resident_range<T>(&self, records: &[T]) -> Result<()> {
        check(unsafe { ffi::iris_device_drop_resident_range(self.raw(), records.as_ptr() as *const c_void) })
    }

    /// Frees every resident file copy of the device (iris_device_drop_resident).
    pub fn drop_resident(&self) -> Result<()> {
        check(unsafe { ffi::iris_device_drop_resident(self.raw()) })
    }
}

static DEFAULT_DEVICE: OnceLock<Device> = OnceLock::new();

/// The process-wide device behind the reference-signature entry points
/// (`arch::dot_bool`, `DistanceEngine::new`, ...), which take no device argument:
/// ordinal `IRIS_HIP_DEVICE` (default 0), opened on first use.  Panics if no
/// gfx950 device can be opened — there is no CPU fallback behind this backend.
pub fn default_device() -> &'static Device {
    DEFAULT_DEVICE.get_or_init(|| {
        let ordinal = std::env::var("IRIS_HIP_DEVICE").ok().and_then(|s| s.parse().ok()).unwrap_or(0);
        Device::open(ordinal).unwrap_or_else(|e| panic!("iris_hip: cannot open device {ordinal}: {e}"))
    })
}

/// Record types a device database can hold: the reference's POD value types, whose
/// bytes are exactly the C ABI's record layouts (bytemuck views, src/bits.rs:13-15,
/// src/encoded_bits.rs:13-15, src/template.rs:11-29).
///
/// # Safety
/// `Self` must be `#[repr(C)]`/`#[repr(transparent)]` with the size of the kind's record.
pub unsafe trait Record: Copy {
    const KIND: c_int;
}

unsafe impl Record for Bits {
    const KIND: c_int = ffi::IRIS_KIND_MASKS;
}
unsafe impl Record for EncodedBits {
    const KIND: c_int = ffi::IRIS_KIND_SHARES;
}
unsafe impl Record for Template {
    const KIND: c_int = ffi::IRIS_KIND_TEMPLATES;
}

/// A device-resident database of one record kind (the GPU's replacement for the
/// mmap'd share / masks files, src/main.rs:389,458).
pub struct Database {
    raw: *mut ffi::IrisDb,
    kind: c_int,
    device: Device,
}

unsafe impl Send for Database {}
unsafe impl Sync for Database {}

impl Database {
    pub fn new<T: Record>(device: &Device, capacity: u64) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_db_create(device.raw(), T::KIND, capacity, &mut raw) })?;
        Ok(Database { raw, kind: T::KIND, device: device.clone() })
    }

    /// As `new` with an explicit device layout (`ffi::IRIS_LAYOUT_*`): e.g.
    /// `IRIS_LAYOUT_LANES` for the VALU popcount kernels.
    pub fn with_layout<T: Record>(device: &Device, capacity: u64, layout: c_int) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_db_create_ex(device.raw(), T::KIND, capacity, layout, &mut raw) })?;
        Ok(Database { raw, kind: T::KIND, device: device.clone() })
    }

    /// The device layout the records are held in (`ffi::IRIS_LAYOUT_*`).
    pub fn layout(&self) -> Result<c_int> {
        let mut l: c_int = 0;
        check(unsafe { ffi::iris_db_layout(self.raw, &mut l) }).map(|_| l)
    }

    pub fn raw(&self) -> *mut ffi::IrisDb {
        self.raw
    }

    pub fn kind(&self) -> c_int {
        self.kind
    }

    pub fn device(&self) -> &Device {
        &self.device
    }

    pub fn len(&self) -> u64 {
        let mut n = 0u64;
        check(unsafe { ffi::iris_db_len(self.raw, &mut n) }).map(|_| n).unwrap_or(0)
    }

    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }

    pub(crate) fn expect_kind<T: Record>(&self) -> Result<()> {
        if T::KIND != self.kind {
            return Err(Error { code: ffi::IRIS_E_ARG, message: "record kind does not match the database".into() });
        }
        Ok(())
    }

    pub fn append<T: Record>(&mut self, records: &[T]) -> Result<()> {
        self.expect_kind::<T>()?;
        check(unsafe { ffi::iris_db_append(self.raw, records.as_ptr().cast(), records.len() as u64) })
    }

    pub fn write<T: Record>(&mut self, index: u64, records: &[T]) -> Result<()> {
        self.expect_kind::<T>()?;
        check(unsafe { ffi::iris_db_write(self.raw, index, records.as_ptr().cast(), records.len() as u64) })
    }

    pub fn read<T: Record>(&self, first: u64, out: &mut [T]) -> Result<()> {
        self.expect_kind::<T>()?;
        check(unsafe { ffi::iris_db_read(self.raw, first, out.len() as u64, out.as_mut_ptr().cast()) })
    }

    /// Appends records [first, first + count) of a raw record file (`.masks`,
    /// `.share-i`, raw templates; `count = u64::MAX`: to the end).  A file that is not
    /// a whole number of records is rejected like the reference's `try_cast_slice`.
    pub fn load_file(&mut self, path: &Path, first: u64, count: u64) -> Result<u64> {
        let c = path_cstring(path)?;
        let mut loaded = 0u64;
        check(unsafe { ffi::iris_db_load_file(self.raw, c.as_ptr(), first, count, &mut loaded) })?;
        Ok(loaded)
    }

    pub fn save_file(&self, path: &Path, first: u64, n: u64) -> Result<()> {
        let c = path_cstring(path)?;
        check(unsafe { ffi::iris_db_save_file(self.raw, c.as_ptr(), first, n) })
    }
}

impl Drop for Database {
    fn drop(&mut self) {
        unsafe {
            ffi::iris_db_destroy(self.raw);
        }
    }
}

/// A `Database` that is the device copy of a host record array — typically the
/// participant's or resolver's memory-mapped record file (src/main.rs:389-391,
/// 458-460).  While it lives, the reference-signature calls
/// `DistanceEngine::batch_process(out, chunk)` / `MasksEngine::batch_process(out, chunk)`
/// on any sub-slice `chunk` of that array (the 20 000-record loop of src/main.rs:428-431,
/// 513-516) run on the resident copy and upload nothing (`iris_db_attach_host`).  The
/// borrow keeps the array alive and unchanged; dropping this detaches and frees the
/// device copy.
pub struct AttachedDatabase<'a> {
    db: Database,
    _host: PhantomData<&'a [u8]>,
}

impl<'a> AttachedDatabase<'a> {
    /// Uploads `records` into a new database on `device` and attaches it.
    pub fn new<T: Record>(device: &Device, records: &'a [T]) -> Result<Self> {
        let db = Database::new::<T>(device, records.len() as u64)?;
        check(unsafe { ffi::iris_db_attach_host(db.raw, records.as_ptr().cast(), records.len() as u64, 1) })?;
        Ok(AttachedDatabase { db, _host: PhantomData })
    }

    /// Attaches a database that already holds exactly `records` (e.g. loaded from the
    /// same file with `Database::load_file`; its first, middle and last record are checked).
    pub fn from_loaded<T: Record>(db: Database, records: &'a [T]) -> Result<Self> {
        db.expect_kind::<T>()?;
        check(unsafe { ffi::iris_db_attach_host(db.raw, records.as_ptr().cast(), records.len() as u64, 0) })?;
        Ok(AttachedDatabase { db, _host: PhantomData })
    }

    /// The resident database (device-resident engine forms, searches).
    pub fn database(&self) -> &Database {
        &self.db
    }

    /// Ends the attachment and returns the database.
    pub fn into_inner(self) -> Database {
        unsafe {
            ffi::iris_db_detach_host(self.db.raw);
        }
        let me = std::mem::ManuallyDrop::new(self);
        unsafe { ptr::read(&me.db) }
    }
}

impl Drop for AttachedDatabase<'_> {
    fn drop(&mut self) {
        unsafe {
            ffi::iris_db_detach_host(self.db.raw);
        }
    }
}

/// Devices searched together (`iris_group_*`): the multi-GPU form of the resolver's
/// fan-out and sequential minimum (src/main.rs:486-504, 616-621).  A template database is
/// split into contiguous shards, every device searches its own, and the per-shard winners
/// are all-gathered by the library's RCCL communicator and merged on every device.
pub struct Group {
    raw: *mut ffi::IrisGroup,
}

unsafe impl Send for Group {}
unsafe impl Sync for Group {}

impl Group {
    /// One process driving `ordinals` (ncclCommInitAll).
    pub fn new(ordinals: &[i32]) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_group_create(ordinals.as_ptr(), ordinals.len() as u32, &mut raw) })?;
        Ok(Group { raw })
    }

    /// The 128-byte id rank 0 creates and every rank of a multi-process group joins with.
    pub fn unique_id() -> Result<[u8; ffi::IRIS_GROUP_ID_BYTES]> {
        let mut id = [0u8; ffi::IRIS_GROUP_ID_BYTES];
        check(unsafe { ffi::iris_group_unique_id(id.as_mut_ptr()) })?;
        Ok(id)
    }

    /// This process's one device as `rank` of `nranks` (ncclCommInitRank).
    pub fn rank(ordinal: i32, nranks: u32, rank: u32, id: &[u8; ffi::IRIS_GROUP_ID_BYTES]) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { ffi::iris_group_create_rank(ordinal, nranks, rank, id.as_ptr(), &mut raw) })?;
        Ok(Group { raw })
    }

    /// (local devices, ranks in the group, rank of local device 0).
    pub fn info(&self) -> Result<(u32, u32, u32)> {
        let (mut l, mut r, mut f) = (0u32, 0u32, 0u32);
        check(unsafe { ffi::iris_group_info(self.raw, &mut l, &mut r, &mut f) })?;
        Ok((l, r, f))
    }

    /// Bound of the exchange waits of later calls in milliseconds (0: automatic). A wait that
    /// runs out aborts the group's communicators and returns `Err`; the group then refuses
    /// further calls (include/iris_hip.h, "device groups").
    pub fn set_timeout(&self, ms: u32) -> Result<()> {
        check(unsafe { ffi::iris_group_set_timeout(self.raw, ms) })
    }
}

impl Drop for Group {
    fn drop(&mut self) {
        unsafe {
            ffi::iris_group_destroy(self.raw);
        }
    }
}

/// `total` templates in S = ranks x `shards_per_device` contiguous shards over a `Group`
/// (shard s holds global records [s*total/S, (s+1)*total/S)); records start empty.
pub struct ShardedDatabase {
    raw: *mut ffi::IrisGroupDb,
}

unsafe impl Send for ShardedDatabase {}
unsafe impl Sync for ShardedDatabase {}

/// An enqueued group search; `wait` blocks for it alone.
pub struct PendingShardedSearch {
    raw: *mut ffi::IrisGroupPending,
}

unsafe impl Send for PendingShardedSearch {}

impl PendingShardedSearch {
    pub fn wait(mut self) -> Result<(f64, usize)> {
        let mut m = ffi::IrisMatch::default();
        let raw = std::mem::replace(&mut self.raw, ptr::null_mut());
        check(unsafe { ffi::iris_group_pending_wait(raw, &mut m) })?;
        Ok(match_to_pair(&m))
    }
}

impl Drop for PendingShardedSearch {
    fn drop(&mut self) {
        if !self.raw.is_null() {
            let mut m = ffi::IrisMatch::default();
            unsafe {
                ffi::iris_group_pending_wait(self.raw, &mut m);
            }
        }
    }
}

impl ShardedDatabase {
    pub fn new(group: &Group, total: u64, layout: c_int, shards_per_device: u32) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe {
            ffi::iris_group_db_create(group.raw, ffi::IRIS_KIND_TEMPLATES, total, layout, shards_per_device, &mut raw)
        })?;
        Ok(ShardedDatabase { raw })
    }

    pub fn raw(&self) -> *mut ffi::IrisGroupDb {
        self.raw
    }

    /// Writes global records [index, index + records.len()) (this process's part of them).
    pub fn write(&mut self, index: u64, records: &[Template]) -> Result<()> {
        check(unsafe { ffi::iris_group_db_write(self.raw, index, records.as_ptr().cast(), records.len() as u64) })
    }

    pub fn read(&self, index: u64, out: &mut [Template]) -> Result<()> {
        check(unsafe { ffi::iris_group_db_read(self.raw, index, out.len() as u64, out.as_mut_ptr().cast()) })
    }

    /// Global record i <- record first + i of a raw template file (local shards, in parallel).
    pub fn load_file(&mut self, path: &Path, first: u64) -> Result<()> {
        let c = path_cstring(path)?;
        check(unsafe { ffi::iris_group_db_load_file(self.raw, c.as_ptr(), first) })
    }

    /// The resolver's `(min_distance, min_index)` of `query` over every shard, bit-exact
    /// with `Template::distance` and the strict-< scan (src/template.rs:43-64, src/main.rs:616-621).
    pub fn search(&self, query: &Template) -> Result<(f64, usize)> {
        let mut m = ffi::IrisMatch::default();
        let q = query as *const Template as *const ffi::IrisTemplate;
        check(unsafe { ffi::iris_group_template_search(self.raw, q, &mut m) })?;
        Ok(match_to_pair(&m))
    }

    pub fn search_async(&self, query: &Template) -> Result<PendingShardedSearch> {
        let mut raw = ptr::null_mut();
        let q = query as *const Template as *const ffi::IrisTemplate;
        check(unsafe { ffi::iris_group_template_search_async(self.raw, q, &mut raw) })?;
        Ok(PendingShardedSearch { raw })
    }

    pub fn batch_search(&self, queries: &[Template]) -> Result<Vec<(f64, usize)>> {
        let mut out = vec![ffi::IrisMatch::default(); queries.len()];
        check(unsafe {
            ffi::iris_group_template_batch_search(self.raw, queries.as_ptr().cast(), queries.len() as u32, out.as_mut_ptr())
        })?;
        Ok(out.iter().map(match_to_pair).collect())
    }
}

impl Drop for ShardedDatabase {
    fn drop(&mut self) {
        unsafe {
            ffi::iris_group_db_destroy(self.raw);
        }
    }
}

fn path_cstring(path: &Path) -> Result<CString> {
    use std::os::unix::ffi::OsStrExt;
    CString::new(path.as_os_str().as_bytes())
        .map_err(|_| Error { code: ffi::IRIS_E_ARG, message: "path contains a NUL byte".into() })
}

/// `(min_distance, min_index)` as the reference's resolver reports them
/// (src/main.rs:581-582, 616-621): `usize::MAX` and +inf when nothing matched.
pub fn match_to_pair(m: &ffi::IrisMatch) -> (f64, usize) {
    let index = if m.index == u64::MAX { usize::MAX } else { m.index as usize };
    (m.distance, index)
}

/// The resolver's aggregation (src/main.rs:597-621) over host arrays: wrapping sum
/// of every participant's `[u16; 31]`, `decode_distance`, first strict minimum.
pub fn resolver_search(shares: &[&[[u16; 31]]], denominators: &[[u16; 31]]) -> (f64, usize) {
    for s in shares {
        assert_eq!(s.len(), denominators.len());
    }
    let ptrs: Vec<*const u16> = shares.iter().map(|s| s.as_ptr().cast::<u16>()).collect();
    let mut m = ffi::IrisMatch::default();
    check(unsafe {
        ffi::iris_resolver_search_host(
            default_device().raw(),
            ptrs.as_ptr(),
            ptrs.len() as u32,
            denominators.as_ptr().cast(),
            denominators.len() as u64,
            0,
            &mut m,
        )
    })
    .unwrap_or_else(|e| panic!("resolver_search: {e}"));
    match_to_pair(&m)
}
