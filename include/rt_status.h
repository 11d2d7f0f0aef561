/*
 * rt_status.h -- status codes of the C ABIs.
 *
 * Same numbers and meaning as the cl_int codes the reference surfaces through
 * CLException (CLutils.h:11-105 GetClErrorString, :107-114).  0 = success.
 */
#ifndef RT_STATUS_H
#define RT_STATUS_H

#define RT_SUCCESS 0
#define RT_DEVICE_NOT_FOUND (-1)
#define RT_MEM_OBJECT_ALLOCATION_FAILURE (-4)
#define RT_OUT_OF_RESOURCES (-5)
#define RT_OUT_OF_HOST_MEMORY (-6)
#define RT_INVALID_VALUE (-30)
#define RT_INVALID_DEVICE (-33)
#define RT_INVALID_CONTEXT (-34)
#define RT_INVALID_COMMAND_QUEUE (-36)
#define RT_INVALID_HOST_PTR (-37)
#define RT_INVALID_MEM_OBJECT (-38)
#define RT_INVALID_KERNEL_NAME (-46)
#define RT_INVALID_KERNEL (-48)
#define RT_INVALID_ARG_INDEX (-49)
#define RT_INVALID_ARG_VALUE (-50)
#define RT_INVALID_ARG_SIZE (-51)
#define RT_INVALID_KERNEL_ARGS (-52)
#define RT_INVALID_GLOBAL_WORK_SIZE (-63)
#define RT_INVALID_OPERATION (-59)
#define RT_INVALID_BUFFER_SIZE (-61)
/* scene pipeline (host) */
#define RT_FILE_NOT_FOUND (-1001)
#define RT_PARSE_ERROR (-1002)

/* Mirrors GetClErrorString (CLutils.h:31-105) for the codes above. */
static inline const char* rtGetErrorString(int code) {
    switch (code) {
        case RT_SUCCESS: return "CL_SUCCESS";
        case RT_DEVICE_NOT_FOUND: return "CL_DEVICE_NOT_FOUND";
        case RT_MEM_OBJECT_ALLOCATION_FAILURE: return "CL_MEM_OBJECT_ALLOCATION_FAILURE";
        case RT_OUT_OF_RESOURCES: return "CL_OUT_OF_RESOURCES";
        case RT_OUT_OF_HOST_MEMORY: return "CL_OUT_OF_HOST_MEMORY";
        case RT_INVALID_VALUE: return "CL_INVALID_VALUE";
        case RT_INVALID_DEVICE: return "CL_INVALID_DEVICE";
        case RT_INVALID_CONTEXT: return "CL_INVALID_CONTEXT";
        case RT_INVALID_COMMAND_QUEUE: return "CL_INVALID_COMMAND_QUEUE";
        case RT_INVALID_HOST_PTR: return "CL_INVALID_HOST_PTR";
        case RT_INVALID_MEM_OBJECT: return "CL_INVALID_MEM_OBJECT";
        case RT_INVALID_KERNEL_NAME: return "CL_INVALID_KERNEL_NAME";
        case RT_INVALID_KERNEL: return "CL_INVALID_KERNEL";
        case RT_INVALID_ARG_INDEX: return "CL_INVALID_ARG_INDEX";
        case RT_INVALID_ARG_VALUE: return "CL_INVALID_ARG_VALUE";
        case RT_INVALID_ARG_SIZE: return "CL_INVALID_ARG_SIZE";
        case RT_INVALID_KERNEL_ARGS: return "CL_INVALID_KERNEL_ARGS";
        case RT_INVALID_GLOBAL_WORK_SIZE: return "CL_INVALID_GLOBAL_WORK_SIZE";
        case RT_INVALID_OPERATION: return "CL_INVALID_OPERATION";
        case RT_INVALID_BUFFER_SIZE: return "CL_INVALID_BUFFER_SIZE";
        case RT_FILE_NOT_FOUND: return "RT_FILE_NOT_FOUND";
        case RT_PARSE_ERROR: return "RT_PARSE_ERROR";
        default: return "Unknown OpenCL error";
    }
}

#endif /* RT_STATUS_H */
