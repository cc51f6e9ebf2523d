//! HIP (MI355X / gfx950) backend for the `arch` plugin point.
//!
//! Drop-in for `src/arch/generic.rs`: the same two functions with the same
//! signatures (src/arch/generic.rs:4,11), so the backend switch at
//! src/arch/mod.rs:5 is the one-word change
//!
//! ```text
//! pub use hip::{dot_bool, dot_u16};
//! ```
//!
//! Both run on the process-wide default device (`crate::iris_hip::default_device`,
//! ordinal `IRIS_HIP_DEVICE`, default 0) through `iris_dot_bool_batch` /
//! `iris_dot_u16_batch` of `include/iris_hip.h`.  A per-pair call is one FFI call
//! and one kernel launch (~10 µs): correct, but launch-bound, exactly as the
//! reference's own per-pair functions are the slow path.  Callers with many pairs
//! use `dot_bool_batch` / `dot_u16_batch` below or the engines
//! (`crate::iris_hip::engines`), which is where the GPU pays.  There is no CPU
//! fallback: without a gfx950 device the first call panics.
#![allow(unused)]
use crate::{
    bits::LIMBS,
    iris_hip::{check, default_device, ffi},
    BITS,
};

/// Σ popcount(a[i] & b[i]) with wrapping u16 adds (src/arch/generic.rs:4-9).
pub fn dot_bool(a: &[u64; LIMBS], b: &[u64; LIMBS]) -> u16 {
    let mut out = 0_u16;
    check(unsafe { ffi::iris_dot_bool_batch(default_device().raw(), a.as_ptr(), 1, b.as_ptr(), 1, &mut out) })
        .unwrap_or_else(|e| panic!("arch::hip::dot_bool: {e}"));
    out
}

/// Σ a[i]·b[i] mod 2^16 (wrapping_mul, wrapping_add; src/arch/generic.rs:11-16).
pub fn dot_u16(a: &[u16; BITS], b: &[u16; BITS]) -> u16 {
    let mut out = 0_u16;
    check(unsafe { ffi::iris_dot_u16_batch(default_device().raw(), a.as_ptr(), 1, b.as_ptr(), 1, &mut out) })
        .unwrap_or_else(|e| panic!("arch::hip::dot_u16: {e}"));
    out
}

/// All pairs in one launch, in the criterion harness's loop order
/// (src/arch/mod.rs:34-41): `out[j * a.len() + i] = dot_bool(&a[i], &b[j])`.
pub fn dot_bool_batch(a: &[[u64; LIMBS]], b: &[[u64; LIMBS]], out: &mut [u16]) {
    assert_eq!(out.len(), a.len() * b.len());
    if out.is_empty() {
        return;
    }
    check(unsafe {
        ffi::iris_dot_bool_batch(
            default_device().raw(),
            a.as_ptr().cast(),
            a.len() as u64,
            b.as_ptr().cast(),
            b.len() as u64,
            out.as_mut_ptr(),
        )
    })
    .unwrap_or_else(|e| panic!("arch::hip::dot_bool_batch: {e}"));
}

/// All pairs in one launch: `out[j * a.len() + i] = dot_u16(&a[i], &b[j])` (src/arch/mod.rs:62-69).
pub fn dot_u16_batch(a: &[[u16; BITS]], b: &[[u16; BITS]], out: &mut [u16]) {
    assert_eq!(out.len(), a.len() * b.len());
    if out.is_empty() {
        return;
    }
    check(unsafe {
        ffi::iris_dot_u16_batch(
            default_device().raw(),
            a.as_ptr().cast(),
            a.len() as u64,
            b.as_ptr().cast(),
            b.len() as u64,
            out.as_mut_ptr(),
        )
    })
    .unwrap_or_else(|e| panic!("arch::hip::dot_u16_batch: {e}"));
}

#[cfg(feature = "bench")]
pub mod benches {
    use super::{
        super::benches::{bench_dot_bool, bench_dot_u16},
        *,
    };
    use criterion::Criterion;

    pub fn group(criterion: &mut Criterion) {
        bench_dot_bool(criterion, "hip/dot_bool", dot_bool);
        bench_dot_u16(criterion, "hip/dot_u16", dot_u16);
    }
}

#[cfg(test)]
mod tests {
    //! Bit-exact against the generic backend, including the wrapping u16 cases the
    //! SVE test probes (src/arch/sve.rs:79-108).
    use super::*;
    use crate::{Bits, EncodedBits};
    use rand::{thread_rng, Rng};

    #[test]
    fn dot_bool_matches_generic() {
        let mut rng = thread_rng();
        for _ in 0..20 {
            let a: Bits = rng.gen();
            let b: Bits = rng.gen();
            assert_eq!(dot_bool(&a.0, &b.0), super::super::generic::dot_bool(&a.0, &b.0));
        }
        let ones = [u64::MAX; LIMBS];
        assert_eq!(dot_bool(&ones, &ones), 12800);
    }

    #[test]
    fn dot_u16_matches_generic() {
        let mut rng = thread_rng();
        for _ in 0..20 {
            let a: EncodedBits = rng.gen();
            let b: EncodedBits = rng.gen();
            assert_eq!(dot_u16(&a.0, &b.0), super::super::generic::dot_u16(&a.0, &b.0));
        }
        let max = [u16::MAX; BITS];
        assert_eq!(dot_u16(&max, &max), super::super::generic::dot_u16(&max, &max));
    }

    #[test]
    fn batch_matches_pairs() {
        let mut rng = thread_rng();
        let a: Vec<[u64; LIMBS]> = (0..3).map(|_| rng.gen::<Bits>().0).collect();
        let b: Vec<[u64; LIMBS]> = (0..5).map(|_| rng.gen::<Bits>().0).collect();
        let mut out = vec![0_u16; 15];
        dot_bool_batch(&a, &b, &mut out);
        for j in 0..5 {
            for i in 0..3 {
                assert_eq!(out[j * 3 + i], super::super::generic::dot_bool(&a[i], &b[j]));
            }
        }
    }
}
