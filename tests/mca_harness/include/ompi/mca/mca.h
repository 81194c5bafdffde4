/* TEST HARNESS ONLY: the component-description fields the glue sets. */
#ifndef HARNESS_MCA_H
#define HARNESS_MCA_H
typedef struct mca_base_component_t {
    int mca_major_version, mca_minor_version, mca_release_version;
    char mca_type_name[32];
    int mca_type_major_version, mca_type_minor_version, mca_type_release_version;
    char mca_component_name[64];
    int mca_component_major_version, mca_component_minor_version, mca_component_release_version;
    int (*mca_open_component)(void);
    int (*mca_close_component)(void);
    int (*mca_query_component)(void);
    int (*mca_register_component_params)(void);
} mca_base_component_t;
typedef struct mca_base_component_data_t { int param_field; } mca_base_component_data_t;
#define OMPI_MCA_BASE_VERSION_2_1_0(type, a, b, c) \
    .mca_major_version = 2, .mca_minor_version = 1, .mca_release_version = 0, \
    .mca_type_name = type, .mca_type_major_version = a, .mca_type_minor_version = b, \
    .mca_type_release_version = c
#define MCA_BASE_MAKE_VERSION(kind, a, b, c) \
    .mca_##kind##_major_version = a, .mca_##kind##_minor_version = b, \
    .mca_##kind##_release_version = c
#define MCA_BASE_METADATA_PARAM_CHECKPOINT .param_field = 1
#endif
