/*! H5Part-compatible HDF5 I/O (serial libhdf5), exposed as the _sphx_io module.
 *
 * Layout (reference extern/h5part/H5Part.c:96,612-626 and main/src/io/h5part_wrapper.hpp:47-344):
 *   /                 file attributes (test-case settings, one value each)
 *   /Step#<n>         one group per output step, step attributes (iteration, time, minDt, ...; box, boundaryType)
 *   /Step#<n>/<field> one 1-D dataset per particle field, global length, ranks' slices concatenated in rank order
 * Type mapping: double->FLOAT64, float->FLOAT32, int32/uint32->INT32, int64/uint64->INT64, char->CHAR.
 * Multi-rank writes are serialized by the caller (rank-ordered hyperslab writes into one pre-sized dataset).
 */
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include <hdf5.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;

namespace
{

void check(herr_t e, const std::string& what)
{
    if (e < 0) throw std::runtime_error("HDF5 error: " + what);
}

hid_t checkId(hid_t id, const std::string& what)
{
    if (id < 0) throw std::runtime_error("HDF5 error: " + what);
    return id;
}

//! dtype code: 'd' f64, 'f' f32, 'i' i32, 'l' i64, 'c' char
hid_t memType(char code)
{
    switch (code)
    {
        case 'd': return H5T_NATIVE_DOUBLE;
        case 'f': return H5T_NATIVE_FLOAT;
        case 'i': return H5T_NATIVE_INT32;
        case 'l': return H5T_NATIVE_INT64;
        case 'c': return H5T_NATIVE_CHAR;
    }
    throw std::runtime_error(std::string("unsupported dtype code ") + code);
}

char codeOf(hid_t type)
{
    H5T_class_t cls = H5Tget_class(type);
    size_t sz       = H5Tget_size(type);
    if (cls == H5T_FLOAT) return sz == 8 ? 'd' : 'f';
    if (cls == H5T_INTEGER) return sz == 8 ? 'l' : (sz == 1 ? 'c' : 'i');
    throw std::runtime_error("unsupported HDF5 type class");
}

char codeOfDtype(const py::dtype& dt)
{
    char k = dt.kind();
    auto sz = dt.itemsize();
    if (k == 'f') return sz == 8 ? 'd' : 'f';
    if (k == 'i' || k == 'u') return sz == 8 ? 'l' : (sz == 1 ? 'c' : 'i');
    if (k == 'b') return 'c';
    throw std::runtime_error("unsupported numpy dtype");
}

py::dtype dtypeOf(char code)
{
    switch (code)
    {
        case 'd': return py::dtype::of<double>();
        case 'f': return py::dtype::of<float>();
        case 'i': return py::dtype::of<int32_t>();
        case 'l': return py::dtype::of<int64_t>();
        case 'c': return py::dtype::of<int8_t>();
    }
    throw std::runtime_error("bad code");
}

std::string stepName(int64_t step) { return "Step#" + std::to_string(step); }

herr_t countSteps(hid_t, const char* name, const H5L_info_t*, void* data)
{
    if (std::strncmp(name, "Step#", 5) == 0) (*static_cast<int64_t*>(data))++;
    return 0;
}

herr_t collectNames(hid_t, const char* name, const H5L_info_t*, void* data)
{
    static_cast<std::vector<std::string>*>(data)->emplace_back(name);
    return 0;
}

herr_t collectAttrNames(hid_t, const char* name, const H5A_info_t*, void* data)
{
    static_cast<std::vector<std::string>*>(data)->emplace_back(name);
    return 0;
}

void writeAttr(hid_t loc, const std::string& name, py::array arr)
{
    char code  = codeOfDtype(arr.dtype());
    hsize_t n  = hsize_t(arr.size());
    if (H5Aexists(loc, name.c_str()) > 0) check(H5Adelete(loc, name.c_str()), "delete attr");
    hid_t space = checkId(H5Screate_simple(1, &n, nullptr), "attr space");
    hid_t attr  = checkId(H5Acreate2(loc, name.c_str(), memType(code), space, H5P_DEFAULT, H5P_DEFAULT), "attr");
    auto c      = py::array::ensure(arr, py::array::c_style);
    check(H5Awrite(attr, memType(code), c.data()), "attr write");
    H5Aclose(attr);
    H5Sclose(space);
}

py::dict readAttrs(hid_t loc)
{
    std::vector<std::string> names;
    hsize_t idx = 0;
    H5Aiterate2(loc, H5_INDEX_CRT_ORDER, H5_ITER_NATIVE, &idx, collectAttrNames, &names);
    if (names.empty())
    {
        idx = 0;
        H5Aiterate2(loc, H5_INDEX_NAME, H5_ITER_NATIVE, &idx, collectAttrNames, &names);
    }
    py::dict d;
    for (auto& n : names)
    {
        hid_t attr  = H5Aopen(loc, n.c_str(), H5P_DEFAULT);
        hid_t ftype = H5Aget_type(attr);
        hid_t space = H5Aget_space(attr);
        hssize_t np = H5Sget_simple_extent_npoints(space);
        char code   = codeOf(ftype);
        py::array out(dtypeOf(code), std::vector<py::ssize_t>{py::ssize_t(np)});
        check(H5Aread(attr, memType(code), out.mutable_data()), "attr read");
        d[py::str(n)] = out;
        H5Sclose(space);
        H5Tclose(ftype);
        H5Aclose(attr);
    }
    return d;
}

} // namespace

PYBIND11_MODULE(_sphx_io, m)
{
    m.doc() = "H5Part-compatible HDF5 I/O";

    m.def("open", [](const std::string& path, const std::string& mode)
          {
              H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr);
              hid_t f;
              if (mode == "w")
              {
                  hid_t fcpl = H5Pcreate(H5P_FILE_CREATE);
                  H5Pset_link_creation_order(fcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED);
                  H5Pset_attr_creation_order(fcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED);
                  f = H5Fcreate(path.c_str(), H5F_ACC_TRUNC, fcpl, H5P_DEFAULT);
                  H5Pclose(fcpl);
              }
              else if (mode == "a") { f = H5Fopen(path.c_str(), H5F_ACC_RDWR, H5P_DEFAULT); }
              else { f = H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT); }
              return int64_t(checkId(f, "open " + path));
          });

    m.def("close", [](int64_t f) { check(H5Fclose(hid_t(f)), "close"); });

    m.def("num_steps", [](int64_t f)
          {
              int64_t cnt = 0;
              hsize_t idx = 0;
              H5Literate(hid_t(f), H5_INDEX_NAME, H5_ITER_NATIVE, &idx, countSteps, &cnt);
              return cnt;
          });

    m.def("create_step", [](int64_t f, int64_t step)
          {
              hid_t gcpl = H5Pcreate(H5P_GROUP_CREATE);
              H5Pset_link_creation_order(gcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED);
              H5Pset_attr_creation_order(gcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED);
              hid_t g = H5Gcreate2(hid_t(f), stepName(step).c_str(), H5P_DEFAULT, gcpl, H5P_DEFAULT);
              H5Pclose(gcpl);
              return int64_t(checkId(g, "create step"));
          });

    m.def("open_step", [](int64_t f, int64_t step)
          { return int64_t(checkId(H5Gopen2(hid_t(f), stepName(step).c_str(), H5P_DEFAULT), "open step")); });

    m.def("close_group", [](int64_t g) { check(H5Gclose(hid_t(g)), "close group"); });

    m.def("root", [](int64_t f)
          { return int64_t(checkId(H5Gopen2(hid_t(f), "/", H5P_DEFAULT), "open root")); });

    m.def("write_attr", [](int64_t loc, const std::string& name, py::array a) { writeAttr(hid_t(loc), name, a); });

    m.def("read_attrs", [](int64_t loc) { return readAttrs(hid_t(loc)); });

    m.def("dataset_names", [](int64_t g)
          {
              std::vector<std::string> names;
              hsize_t idx = 0;
              H5Literate(hid_t(g), H5_INDEX_NAME, H5_ITER_NATIVE, &idx, collectNames, &names);
              return names;
          });

    m.def("dataset_length", [](int64_t g, const std::string& name)
          {
              hid_t ds    = checkId(H5Dopen2(hid_t(g), name.c_str(), H5P_DEFAULT), "open dataset " + name);
              hid_t space = H5Dget_space(ds);
              hssize_t n  = H5Sget_simple_extent_npoints(space);
              H5Sclose(space);
              H5Dclose(ds);
              return int64_t(n);
          });

    m.def("create_dataset", [](int64_t g, const std::string& name, const std::string& code, int64_t total)
          {
              hsize_t n   = hsize_t(total);
              hid_t space = H5Screate_simple(1, &n, nullptr);
              if (H5Lexists(hid_t(g), name.c_str(), H5P_DEFAULT) > 0) H5Ldelete(hid_t(g), name.c_str(), H5P_DEFAULT);
              hid_t ds = checkId(H5Dcreate2(hid_t(g), name.c_str(), memType(code[0]), space, H5P_DEFAULT,
                                            H5P_DEFAULT, H5P_DEFAULT),
                                 "create dataset " + name);
              H5Dclose(ds);
              H5Sclose(space);
          });

    m.def("write_slice", [](int64_t g, const std::string& name, py::array a, int64_t offset)
          {
              auto c      = py::array::ensure(a, py::array::c_style);
              char code   = codeOfDtype(c.dtype());
              hid_t ds    = checkId(H5Dopen2(hid_t(g), name.c_str(), H5P_DEFAULT), "open dataset " + name);
              hid_t fs    = H5Dget_space(ds);
              hsize_t off = hsize_t(offset), cnt = hsize_t(c.size());
              if (cnt > 0)
              {
                  check(H5Sselect_hyperslab(fs, H5S_SELECT_SET, &off, nullptr, &cnt, nullptr), "hyperslab");
                  hid_t ms = H5Screate_simple(1, &cnt, nullptr);
                  check(H5Dwrite(ds, memType(code), ms, fs, H5P_DEFAULT, c.data()), "write " + name);
                  H5Sclose(ms);
              }
              H5Sclose(fs);
              H5Dclose(ds);
          });

    m.def("read_slice", [](int64_t g, const std::string& name, int64_t offset, int64_t count, const std::string& as)
          {
              hid_t ds    = checkId(H5Dopen2(hid_t(g), name.c_str(), H5P_DEFAULT), "open dataset " + name);
              hid_t ftype = H5Dget_type(ds);
              char code   = as.empty() ? codeOf(ftype) : as[0];
              hid_t fs    = H5Dget_space(ds);
              hsize_t off = hsize_t(offset), cnt = hsize_t(count);
              py::array out(dtypeOf(code), std::vector<py::ssize_t>{py::ssize_t(count)});
              if (cnt > 0)
              {
                  check(H5Sselect_hyperslab(fs, H5S_SELECT_SET, &off, nullptr, &cnt, nullptr), "hyperslab");
                  hid_t ms = H5Screate_simple(1, &cnt, nullptr);
                  check(H5Dread(ds, memType(code), ms, fs, H5P_DEFAULT, out.mutable_data()), "read " + name);
                  H5Sclose(ms);
              }
              H5Sclose(fs);
              H5Tclose(ftype);
              H5Dclose(ds);
              return out;
          });

    m.def("flush", [](int64_t f) { H5Fflush(hid_t(f), H5F_SCOPE_GLOBAL); });
}
