"""TEST ONLY: configure's substitution of ompi/include/mpi.h.in, done into a
scratch directory at test time (the reference's file is read in place, the
result is never kept): each `#undef X` of the configure section becomes the
value configure would give an x86-64 Linux gcc build, the others stay
undefined; @OMPI_BEGIN/END_CONFIGURE_SECTION@ markers are dropped."""
import re
import sys

VALUES = {
    "OPAL_BUILD_PLATFORM_COMPILER_FAMILYID": "1", "OPAL_BUILD_PLATFORM_COMPILER_VERSION": "0",
    "OPAL_STDC_HEADERS": "1", "OPAL_HAVE_ATTRIBUTE_DEPRECATED": "1",
    "OPAL_HAVE_ATTRIBUTE_DEPRECATED_ARGUMENT": "1", "OPAL_HAVE_ATTRIBUTE_ERROR": "1",
    "OPAL_HAVE_SYS_TIME_H": "1", "OPAL_HAVE_LONG_LONG": "1", "OPAL_SIZEOF_BOOL": "1",
    "OPAL_SIZEOF_INT": "4", "OPAL_MAX_DATAREP_STRING": "128", "OPAL_MAX_ERROR_STRING": "256",
    "OPAL_MAX_INFO_KEY": "36", "OPAL_MAX_INFO_VAL": "256", "OPAL_MAX_OBJECT_NAME": "64",
    "OPAL_MAX_PORT_NAME": "1024", "OPAL_MAX_PROCESSOR_NAME": "256", "OMPI_ENABLE_MPI1_COMPAT": "0",
    "HAVE_FLOAT__COMPLEX": "1", "HAVE_DOUBLE__COMPLEX": "1", "HAVE_LONG_DOUBLE__COMPLEX": "1",
    "OMPI_MPI_AINT_TYPE": "ptrdiff_t", "OMPI_MPI_OFFSET_TYPE": "long long",
    "OMPI_OFFSET_DATATYPE": "MPI_LONG_LONG", "OMPI_MPI_OFFSET_SIZE": "8",
    "OMPI_MPI_COUNT_TYPE": "long long", "OMPI_PARAM_CHECK": "1",
    "OMPI_WANT_MPI_INTERFACE_WARNING": "0", "OMPI_MAJOR_VERSION": "5", "OMPI_MINOR_VERSION": "0",
    "OMPI_RELEASE_VERSION": "0", "ompi_fortran_bogus_type_t": "int",
    "ompi_fortran_integer_t": "int", "OPAL_C_HAVE_VISIBILITY": "1",
}


def generate(src_path: str, out_path: str) -> None:
    src = open(src_path).read()
    out = re.sub(r"^#undef (\w+)\s*$",
                 lambda m: (f"#define {m.group(1)} {VALUES[m.group(1)]}" if m.group(1) in VALUES
                            else f"/* #undef {m.group(1)} */"), src, flags=re.M)
    out = re.sub(r"@(\w+)@", lambda m: "" if "CONFIGURE_SECTION" in m.group(1) else "0", out)
    with open(out_path, "w") as f:
        f.write(out)


if __name__ == "__main__":
    generate(sys.argv[1], sys.argv[2])
