// nfa_device.h — device building blocks of the NFA kernels.
#pragma once
#include "dewey.h"
#include "interp.h"
#include "java.h"
