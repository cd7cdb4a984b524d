// liblmi_h5.so — HDF5 loaders and the result writer around the hot path
// (include/lmi_h5.h; reference search/search.py:48-49, :79-87 and
// search/li/utils.py:85-97).  Plain C over libhdf5 (1.10, from the image).
#include "../../include/lmi_h5.h"

#include <hdf5.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#define LMI_E_INVALID 1001
#define LMI_E_IO 1005

static __thread char g_err[512];

static int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

const char* lmi_h5_last_error(void) { return g_err; }

static void quiet(void) { H5Eset_auto2(H5E_DEFAULT, NULL, NULL); }

static int32_t classify(hid_t t) {
    const H5T_class_t c = H5Tget_class(t);
    const size_t sz = H5Tget_size(t);
    if (c == H5T_FLOAT) return sz == 4 ? LMI_H5_F32 : sz == 2 ? LMI_H5_F16 : sz == 8 ? LMI_H5_F64 : LMI_H5_OTHER;
    if (c == H5T_INTEGER) {
        const int sgn = H5Tget_sign(t) == H5T_SGN_2;
        if (!sgn && sz == 4) return LMI_H5_U32;
        if (sgn && sz == 8) return LMI_H5_I64;
    }
    return LMI_H5_OTHER;
}

int lmi_h5_dataset_info(const char* path, const char* name, int64_t* dims_out, int32_t* dtype_out) {
    if (!path || !name || !dims_out || !dtype_out) return fail(LMI_E_INVALID, "null argument");
    quiet();
    hid_t f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
    if (f < 0) return fail(LMI_E_IO, "cannot open %s", path);
    int rc = 0;
    hid_t d = H5Dopen2(f, name, H5P_DEFAULT);
    if (d < 0) {
        rc = fail(LMI_E_IO, "%s: no dataset '%s'", path, name);
    } else {
        hid_t sp = H5Dget_space(d), t = H5Dget_type(d);
        hsize_t dims[2] = {0, 1};
        const int rank = H5Sget_simple_extent_ndims(sp);
        if (rank < 1 || rank > 2) {
            rc = fail(LMI_E_INVALID, "%s/%s: rank %d (1 or 2 supported)", path, name, rank);
        } else {
            H5Sget_simple_extent_dims(sp, dims, NULL);
            dims_out[0] = (int64_t)dims[0];
            dims_out[1] = rank == 2 ? (int64_t)dims[1] : 1;
            *dtype_out = classify(t);
        }
        H5Tclose(t);
        H5Sclose(sp);
        H5Dclose(d);
    }
    H5Fclose(f);
    return rc;
}

int lmi_h5_read_f32(const char* path, const char* name, int64_t row0, int64_t nrows, float* out) {
    if (!path || !name || (!out && nrows > 0) || row0 < 0 || nrows < 0)
        return fail(LMI_E_INVALID, "bad argument");
    quiet();
    hid_t f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
    if (f < 0) return fail(LMI_E_IO, "cannot open %s", path);
    int rc = 0;
    hid_t d = H5Dopen2(f, name, H5P_DEFAULT);
    if (d < 0) {
        H5Fclose(f);
        return fail(LMI_E_IO, "%s: no dataset '%s'", path, name);
    }
    hid_t sp = H5Dget_space(d), t = H5Dget_type(d);
    hsize_t dims[2] = {0, 1};
    const int rank = H5Sget_simple_extent_ndims(sp);
    if (rank < 1 || rank > 2 || H5Tget_class(t) != H5T_FLOAT) {
        rc = fail(LMI_E_INVALID, "%s/%s: need a rank-1/2 floating dataset", path, name);
    } else {
        H5Sget_simple_extent_dims(sp, dims, NULL);
        if ((hsize_t)(row0 + nrows) > dims[0]) {
            rc = fail(LMI_E_INVALID, "%s/%s: rows [%lld, %lld) past %llu", path, name,
                      (long long)row0, (long long)(row0 + nrows), (unsigned long long)dims[0]);
        } else if (nrows > 0) {
            hsize_t start[2] = {(hsize_t)row0, 0}, count[2] = {(hsize_t)nrows, rank == 2 ? dims[1] : 1};
            H5Sselect_hyperslab(sp, H5S_SELECT_SET, start, NULL, count, NULL);
            hid_t mem = H5Screate_simple(rank, count, NULL);
            // HDF5 converts the stored IEEE type (f16 / f32 / f64) to native float
            if (H5Dread(d, H5T_NATIVE_FLOAT, mem, sp, H5P_DEFAULT, out) < 0)
                rc = fail(LMI_E_IO, "%s/%s: read failed", path, name);
            H5Sclose(mem);
        }
    }
    H5Tclose(t);
    H5Sclose(sp);
    H5Dclose(d);
    H5Fclose(f);
    return rc;
}

int lmi_h5_read_stored(const char* path, const char* name, int64_t row0, int64_t nrows,
                       int32_t elem_bytes, void* out) {
    if (!path || !name || (!out && nrows > 0) || row0 < 0 || nrows < 0)
        return fail(LMI_E_INVALID, "bad argument");
    quiet();
    hid_t f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
    if (f < 0) return fail(LMI_E_IO, "cannot open %s", path);
    int rc = 0;
    hid_t d = H5Dopen2(f, name, H5P_DEFAULT);
    if (d < 0) {
        H5Fclose(f);
        return fail(LMI_E_IO, "%s: no dataset '%s'", path, name);
    }
    hid_t sp = H5Dget_space(d), t = H5Dget_type(d);
    hsize_t dims[2] = {0, 1};
    const int rank = H5Sget_simple_extent_ndims(sp);
    if (rank < 1 || rank > 2 || (H5Tget_class(t) != H5T_FLOAT && H5Tget_class(t) != H5T_INTEGER) ||
        H5Tget_order(t) != H5T_ORDER_LE) {
        rc = fail(LMI_E_INVALID, "%s/%s: need a rank-1/2 little-endian floating or integer dataset",
                  path, name);
    } else if ((int32_t)H5Tget_size(t) != elem_bytes) {
        rc = fail(LMI_E_INVALID, "%s/%s: stored element is %d bytes, caller expects %d", path, name,
                  (int)H5Tget_size(t), (int)elem_bytes);
    } else {
        H5Sget_simple_extent_dims(sp, dims, NULL);
        if ((hsize_t)(row0 + nrows) > dims[0]) {
            rc = fail(LMI_E_INVALID, "%s/%s: rows [%lld, %lld) past %llu", path, name,
                      (long long)row0, (long long)(row0 + nrows), (unsigned long long)dims[0]);
        } else if (nrows > 0) {
            hsize_t start[2] = {(hsize_t)row0, 0}, count[2] = {(hsize_t)nrows, rank == 2 ? dims[1] : 1};
            H5Sselect_hyperslab(sp, H5S_SELECT_SET, start, NULL, count, NULL);
            hid_t mem = H5Screate_simple(rank, count, NULL);
            // the file's own type as the memory type: the bytes as stored
            // (IEEE binary16 / 32 / 64, little endian), no conversion
            if (H5Dread(d, t, mem, sp, H5P_DEFAULT, out) < 0)
                rc = fail(LMI_E_IO, "%s/%s: read failed", path, name);
            H5Sclose(mem);
        }
    }
    H5Tclose(t);
    H5Sclose(sp);
    H5Dclose(d);
    H5Fclose(f);
    return rc;
}

static int put_str(hid_t obj, const char* key, const char* val) {
    // h5py's Python-str attribute: scalar, variable-length UTF-8
    hid_t t = H5Tcopy(H5T_C_S1);
    H5Tset_size(t, H5T_VARIABLE);
    H5Tset_cset(t, H5T_CSET_UTF8);
    hid_t sp = H5Screate(H5S_SCALAR);
    hid_t a = H5Acreate2(obj, key, t, sp, H5P_DEFAULT, H5P_DEFAULT);
    const char* v = val ? val : "";
    const int ok = a >= 0 && H5Awrite(a, t, &v) >= 0;
    if (a >= 0) H5Aclose(a);
    H5Sclose(sp);
    H5Tclose(t);
    return ok ? 0 : -1;
}

static int put_f64(hid_t obj, const char* key, double val) {
    hid_t sp = H5Screate(H5S_SCALAR);
    hid_t a = H5Acreate2(obj, key, H5T_IEEE_F64LE, sp, H5P_DEFAULT, H5P_DEFAULT);
    const int ok = a >= 0 && H5Awrite(a, H5T_NATIVE_DOUBLE, &val) >= 0;
    if (a >= 0) H5Aclose(a);
    H5Sclose(sp);
    return ok ? 0 : -1;
}

static int put_2d(hid_t f, const char* name, hid_t ftype, hid_t mtype, int64_t nq, int32_t k,
                  const void* buf) {
    hsize_t dims[2] = {(hsize_t)nq, (hsize_t)k};
    hid_t sp = H5Screate_simple(2, dims, NULL);
    hid_t d = H5Dcreate2(f, name, ftype, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    const int ok = d >= 0 && (nq == 0 || k == 0 || H5Dwrite(d, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf) >= 0);
    if (d >= 0) H5Dclose(d);
    H5Sclose(sp);
    return ok ? 0 : -1;
}

int lmi_h5_write_results(const char* path, const uint32_t* knns, const double* dists, int64_t nq,
                         int32_t k, const char* algo, const char* data, double buildtime,
                         double querytime, const char* size, const char* params) {
    if (!path || nq < 0 || k < 0 || ((!knns || !dists) && nq * k > 0))
        return fail(LMI_E_INVALID, "bad argument");
    quiet();
    hid_t f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    if (f < 0) return fail(LMI_E_IO, "cannot create %s", path);
    int bad = 0;
    // the order of utils.py:90-97
    bad |= put_str(f, "algo", algo);
    bad |= put_str(f, "data", data);
    bad |= put_f64(f, "buildtime", buildtime);
    bad |= put_f64(f, "querytime", querytime);
    bad |= put_str(f, "size", size);
    bad |= put_str(f, "params", params);
    bad |= put_2d(f, "knns", H5T_STD_U32LE, H5T_NATIVE_UINT32, nq, k, knns);
    bad |= put_2d(f, "dists", H5T_IEEE_F64LE, H5T_NATIVE_DOUBLE, nq, k, dists);
    if (H5Fclose(f) < 0) bad = 1;
    return bad ? fail(LMI_E_IO, "%s: write failed", path) : 0;
}

int lmi_h5_write_f32(const char* path, const char* name, int32_t dtype, int64_t rows, int64_t cols,
                     const float* buf, int32_t append) {
    if (!path || !name || rows < 0 || cols < 1 || (!buf && rows > 0) ||
        (dtype != LMI_H5_F16 && dtype != LMI_H5_F32))
        return fail(LMI_E_INVALID, "bad argument");
    quiet();
    hid_t f = append ? H5Fopen(path, H5F_ACC_RDWR, H5P_DEFAULT)
                     : H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    if (f < 0) return fail(LMI_E_IO, "cannot %s %s", append ? "open" : "create", path);
    hid_t ft = H5T_IEEE_F32LE, own = -1;
    if (dtype == LMI_H5_F16) {
        // IEEE binary16: 1 sign, 5 exponent (bias 15), 10 mantissa bits
        own = H5Tcopy(H5T_IEEE_F32LE);
        H5Tset_fields(own, 15, 10, 5, 0, 10);
        H5Tset_size(own, 2);
        H5Tset_ebias(own, 15);
        ft = own;
    }
    hsize_t dims[2] = {(hsize_t)rows, (hsize_t)cols};
    hid_t sp = H5Screate_simple(2, dims, NULL);
    hid_t d = H5Dcreate2(f, name, ft, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    const int ok = d >= 0 && (rows == 0 || H5Dwrite(d, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf) >= 0);
    if (d >= 0) H5Dclose(d);
    H5Sclose(sp);
    if (own >= 0) H5Tclose(own);
    if (H5Fclose(f) < 0 || !ok) return fail(LMI_E_IO, "%s/%s: write failed", path, name);
    return 0;
}

int lmi_h5_write_stored(const char* path, const char* name, int32_t elem_bytes, int64_t rows,
                        int64_t cols, const void* buf, int32_t append) {
    if (!path || !name || rows < 0 || cols < 1 || (!buf && rows > 0) ||
        (elem_bytes != 2 && elem_bytes != 4 && elem_bytes != 8))
        return fail(LMI_E_INVALID, "bad argument");
    quiet();
    hid_t f = append ? H5Fopen(path, H5F_ACC_RDWR, H5P_DEFAULT)
                     : H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    if (f < 0) return fail(LMI_E_IO, "cannot %s %s", append ? "open" : "create", path);
    hid_t ft = elem_bytes == 8 ? H5T_IEEE_F64LE : H5T_IEEE_F32LE, own = -1;
    if (elem_bytes == 2) {  // IEEE binary16, as lmi_h5_write_f32 lays it out
        own = H5Tcopy(H5T_IEEE_F32LE);
        H5Tset_fields(own, 15, 10, 5, 0, 10);
        H5Tset_size(own, 2);
        H5Tset_ebias(own, 15);
        ft = own;
    }
    hsize_t dims[2] = {(hsize_t)rows, (hsize_t)cols};
    hid_t sp = H5Screate_simple(2, dims, NULL);
    hid_t d = H5Dcreate2(f, name, ft, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    // the memory type is the file type: the bytes go out unconverted
    const int ok = d >= 0 && (rows == 0 || H5Dwrite(d, ft, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf) >= 0);
    if (d >= 0) H5Dclose(d);
    H5Sclose(sp);
    if (own >= 0) H5Tclose(own);
    if (H5Fclose(f) < 0 || !ok) return fail(LMI_E_IO, "%s/%s: write failed", path, name);
    return 0;
}
